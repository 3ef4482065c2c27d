// tools/small_batch_probe.hip -- fixed per-launch cost of the streaming kernels at the
// per-GPU shares a fixed batch gives under strong scaling (not product).
//
// The RS(3,2) 4 KiB encode at 8,192 stripes (one GPU's share of 65,536 over 8) takes
// about 4 us more than 1/8 of the whole batch, the decode about 2 us.  This streams
// the same shapes as XOR kernels (encode 3 reads / 2 writes, decode 3 reads / 1 write;
// 64-lane workgroups, 16 B per lane, nt loads) alternating encode / decode back to back
// like bench.py's step, with an event between launches, at 8,192 / 16,384 / 65,536
// stripes, for each store policy:
//   nt      __builtin_nontemporal_store (the library's)
//   plain   raw buffer store, aux 0
//   sc1     raw buffer store, aux 16 (write-through: the line leaves the XCD's L2)
//   sc1nt   raw buffer store, aux 18
// and prints per size and policy the median encode / decode us and, per policy, the
// fixed cost a of t(stripes) = a + b * stripes fitted from 8,192 and 65,536.
// `small_batch_probe.bin STEPS loads`: the load policy instead, with write-through stores
// (the library's store at these shares): does a load that may allocate in the
// memory-side cache let the decode re-read what the encode just read / wrote (the whole
// working set of an 8,192-stripe share is 256 MiB)?  Loads: nt (the library's), or a raw
// buffer load with aux 0 (default), 1 (sc0), 16 (sc1), 17 (sc0 sc1).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/small_batch_probe.hip -o tools/small_batch_probe.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t ck_ = (x);                                                \
        if (ck_ != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(ck_));         \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GL __attribute__((address_space(1)))

struct Args {
    const uint8_t *r[3];
    uint8_t *w[2];
    uint32_t bytes;  // per arena (buffer descriptors' range)
};

// `small_batch_probe.bin STEPS kernarg`: the library's kernel-argument form at these shares.
// BigArgs is as large as the library's (48 stream slots + table pointers, 440 B);
// kMode 3 reads its streams at fixed slots, kMode 4 through slot numbers loaded from a
// small table in global memory first (the library's tile -> pattern -> stream chain).
struct BigArgs {
    uint8_t *base[48];
    const uint8_t *slots;  // kMode 4: in slots 0-2, out slots 3-4
    uint64_t pad[6];
    uint32_t bytes;
};

template <int AUX>
__device__ inline void store16(uint8_t *base, uint32_t bytes, uint32_t off, u32x4 v) {
    if constexpr (AUX < 0) {
        __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)base + off));
    } else {
        auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, AUX);
    }
}

// kMode 1: a cold path of byte copies the launch never takes; it only makes the kernel's
// code as large as the library's, to see whether code size (instruction-cache warm-up at
// the start of a launch) is a per-launch cost.  kMode 2: no cold path, but every load
// and nt store through a 64-bit vector address instead of a scalar base + 32-bit vector
// offset (what kMode 1's hot path compiled to), to separate the addressing form.
template <int LAUX>
__device__ inline u32x4 load16(const uint8_t *base, uint32_t bytes, uint32_t off) {
    if constexpr (LAUX < 0) {
        return __builtin_nontemporal_load((const GL u32x4 *)((uintptr_t)base + off));
    } else {
        auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), 0, bytes, 0x00020000);
        return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LAUX);
    }
}

template <int W, int AUX, int kMode = 0, int LAUX = -1>
__global__ __launch_bounds__(64) void k_stream(Args a) {
    const uint32_t off = blockIdx.x * 1024u + threadIdx.x * 16u;
    u32x4 acc = {0, 0, 0, 0};
    if constexpr (kMode == 1) {
        if (blockIdx.x == 0xffffffffu) {  // never: the id is already in an SGPR, no wait
            // byte copies one at a time (the empty asm keeps them from being batched, so
            // the register count stays the fast variant's; only the code grows)
#pragma unroll
            for (int b = 0; b < 240; ++b) {
                const uint8_t v = *(const GL uint8_t *)((uintptr_t)a.r[b % 3] + off + (b * 7919u) % 4096u);
                *(GL uint8_t *)((uintptr_t)a.w[b & 1] + off + (b * 104729u) % 4096u) = (uint8_t)(v ^ b);
                asm volatile("" ::: "memory");
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if constexpr (LAUX >= 0) {
            acc ^= load16<LAUX>(a.r[i], a.bytes, off);
        } else {
            const GL u32x4 *p = (const GL u32x4 *)((uintptr_t)a.r[i] + off);
            if constexpr (kMode == 2) asm volatile("" : "+v"(p));
            acc ^= __builtin_nontemporal_load(p);
        }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
        u32x4 v = acc;
        v.x ^= j;
        if constexpr (kMode == 2 && AUX < 0) {
            GL u32x4 *q = (GL u32x4 *)((uintptr_t)a.w[j] + off);
            asm volatile("" : "+v"(q));
            __builtin_nontemporal_store(v, q);
        } else {
            store16<AUX>(a.w[j], a.bytes, off, v);
        }
    }
}

template <int W, int kMode>
__global__ __launch_bounds__(64) void k_stream_big(BigArgs a) {
    const uint32_t off = blockIdx.x * 1024u + threadIdx.x * 16u;
    int si[5] = {0, 1, 2, 3, 4};
    if constexpr (kMode == 4) {
        const __attribute__((address_space(4))) uint8_t *t =
            (const __attribute__((address_space(4))) uint8_t *)(uintptr_t)a.slots;
#pragma unroll
        for (int i = 0; i < 5; ++i) si[i] = t[i];
    }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 3; ++i)
        acc ^= __builtin_nontemporal_load((const GL u32x4 *)((uintptr_t)a.base[si[i]] + off));
#pragma unroll
    for (int j = 0; j < W; ++j) {
        u32x4 v = acc;
        v.x ^= j;
        store16<16>(a.base[si[3 + j]], a.bytes, off, v);
    }
}

template <int kMode>
static void run_big(const char *name, uint8_t *const *ar, const uint8_t *d_slots_enc,
                    const uint8_t *d_slots_dec, int steps) {
    const uint32_t sizes[] = {8192, 16384, 65536};
    for (uint32_t stripes : sizes) {
        const uint32_t bytes = stripes * 4096u;
        BigArgs enc{}, dec{};
        // slot layout as the library's: data 0-2, parity 3-4, rebuilt 5
        for (int i = 0; i < 6; ++i) enc.base[i] = dec.base[i] = ar[i];
        enc.slots = d_slots_enc;
        dec.slots = d_slots_dec;
        enc.bytes = dec.bytes = bytes;
        if (kMode == 3) {  // fixed slots: the decode reads 1, 2, 3 and writes 5
            dec.base[0] = ar[1]; dec.base[1] = ar[2]; dec.base[2] = ar[3]; dec.base[3] = ar[5];
        }
        const dim3 grid(stripes * 4);
        std::vector<hipEvent_t> ev(2 * steps + 1);
        for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        for (int w = 0; w < 3; ++w) {
            k_stream_big<2, kMode><<<grid, 64>>>(enc);
            k_stream_big<1, kMode><<<grid, 64>>>(dec);
        }
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(ev[0], 0));
        for (int s = 0; s < steps; ++s) {
            k_stream_big<2, kMode><<<grid, 64>>>(enc);
            CK(hipEventRecord(ev[2 * s + 1], 0));
            k_stream_big<1, kMode><<<grid, 64>>>(dec);
            CK(hipEventRecord(ev[2 * s + 2], 0));
        }
        CK(hipDeviceSynchronize());
        std::vector<float> te(steps), td(steps);
        for (int s = 0; s < steps; ++s) {
            CK(hipEventElapsedTime(&te[s], ev[2 * s], ev[2 * s + 1]));
            CK(hipEventElapsedTime(&td[s], ev[2 * s + 1], ev[2 * s + 2]));
        }
        std::sort(te.begin(), te.end());
        std::sort(td.begin(), td.end());
        printf("{\"policy\": \"%s\", \"stripes\": %u, \"encode_us\": %.2f, \"decode_us\": %.2f}\n", name,
               stripes, 1e3 * te[steps / 2], 1e3 * td[steps / 2]);
        for (auto &e : ev) CK(hipEventDestroy(e));
    }
}

__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

template <int AUX, int kMode = 0, int LAUX = -1>
static void run(const char *name, uint8_t *const *ar, uint64_t stride, int steps, double fit[2][2]) {
    const uint32_t sizes[] = {8192, 16384, 65536};
    for (uint32_t stripes : sizes) {
        const uint32_t bytes = stripes * 4096u;
        Args enc{{ar[0], ar[1], ar[2]}, {ar[3], ar[4]}, bytes};
        Args dec{{ar[1], ar[2], ar[3]}, {ar[5], ar[5]}, bytes};
        const dim3 grid(stripes * 4);
        std::vector<hipEvent_t> ev(2 * steps + 1);
        for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        for (int w = 0; w < 3; ++w) {
            k_stream<2, AUX, kMode, LAUX><<<grid, 64>>>(enc);
            k_stream<1, AUX, kMode, LAUX><<<grid, 64>>>(dec);
        }
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(ev[0], 0));
        for (int s = 0; s < steps; ++s) {
            k_stream<2, AUX, kMode, LAUX><<<grid, 64>>>(enc);
            CK(hipEventRecord(ev[2 * s + 1], 0));
            k_stream<1, AUX, kMode, LAUX><<<grid, 64>>>(dec);
            CK(hipEventRecord(ev[2 * s + 2], 0));
        }
        CK(hipDeviceSynchronize());
        std::vector<float> te(steps), td(steps);
        for (int s = 0; s < steps; ++s) {
            CK(hipEventElapsedTime(&te[s], ev[2 * s], ev[2 * s + 1]));
            CK(hipEventElapsedTime(&td[s], ev[2 * s + 1], ev[2 * s + 2]));
        }
        std::sort(te.begin(), te.end());
        std::sort(td.begin(), td.end());
        const double e_us = 1e3 * te[steps / 2], d_us = 1e3 * td[steps / 2];
        const double e_tbs = 5.0 * bytes / (e_us * 1e-6) / 1e12, d_tbs = 4.0 * bytes / (d_us * 1e-6) / 1e12;
        printf("{\"policy\": \"%s\", \"stripes\": %u, \"encode_us\": %.2f, \"decode_us\": %.2f, "
               "\"encode_TBps\": %.3f, \"decode_TBps\": %.3f}\n",
               name, stripes, e_us, d_us, e_tbs, d_tbs);
        if (stripes == 8192) { fit[0][0] = e_us; fit[1][0] = d_us; }
        if (stripes == 65536) { fit[0][1] = e_us; fit[1][1] = d_us; }
        for (auto &e : ev) CK(hipEventDestroy(e));
    }
    // t = a + b * stripes through (8192, t8) and (65536, t64)
    for (int op = 0; op < 2; ++op) {
        const double b = (fit[op][1] - fit[op][0]) / (65536.0 - 8192.0), a = fit[op][0] - b * 8192.0;
        printf("{\"policy\": \"%s\", \"op\": \"%s\", \"fixed_us\": %.2f, \"us_per_1k_stripes\": %.3f, "
               "\"strong8_efficiency\": %.4f}\n",
               name, op ? "decode" : "encode", a, b * 1024, fit[op][1] / (8.0 * fit[op][0]));
    }
    (void)stride;
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t len = 65536ull * 4096;
    uint64_t stride = (len + 4095) / 4096;
    if (stride % 2 == 0) ++stride;  // the library's odd-4 KiB arena stride
    stride *= 4096;
    uint8_t *slab;
    CK(hipMalloc(&slab, stride * 6));
    uint8_t *ar[6];
    for (int i = 0; i < 6; ++i) {
        ar[i] = slab + i * stride;
        k_fill<<<4096, 256>>>((uint64_t *)ar[i], len / 8, 0xC0C70000ull + i);
    }
    CK(hipDeviceSynchronize());
    double fit[2][2];
    const bool loads = argc > 2 && !strcmp(argv[2], "loads");
    if (argc > 2 && !strcmp(argv[2], "kernarg")) {
        const uint8_t h_enc[8] = {0, 1, 2, 3, 4, 0, 0, 0}, h_dec[8] = {1, 2, 3, 5, 5, 0, 0, 0};
        uint8_t *d_slots;
        CK(hipMalloc(&d_slots, 16));
        CK(hipMemcpy(d_slots, h_enc, 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_slots + 8, h_dec, 8, hipMemcpyHostToDevice));
        double fit[2][2];
        for (int rep = 0; rep < 3; ++rep) {
            run<16>("sc1", ar, stride, steps, fit);
            run_big<3>("sc1_bigargs", ar, d_slots, d_slots + 8, steps);
            run_big<4>("sc1_bigargs_slot_table", ar, d_slots, d_slots + 8, steps);
        }
        CK(hipFree(d_slots));
        CK(hipFree(slab));
        return 0;
    }
    for (int rep = 0; loads && rep < 3; ++rep) {
        run<16, 0, -1>("sc1_ld_nt", ar, stride, steps, fit);
        run<16, 0, 0>("sc1_ld_plain", ar, stride, steps, fit);
        run<16, 0, 1>("sc1_ld_sc0", ar, stride, steps, fit);
        run<16, 0, 16>("sc1_ld_sc1", ar, stride, steps, fit);
        run<16, 0, 17>("sc1_ld_sc0sc1", ar, stride, steps, fit);
        run<-1, 0, 0>("nt_ld_plain", ar, stride, steps, fit);
    }
    for (int rep = 0; !loads && rep < 2; ++rep) {  // two passes: policy order effects show up
        run<-1>("nt", ar, stride, steps, fit);
        run<0>("plain", ar, stride, steps, fit);
        run<16>("sc1", ar, stride, steps, fit);
        run<18>("sc1nt", ar, stride, steps, fit);
        run<16, 1>("sc1_bigcode", ar, stride, steps, fit);
        run<-1, 1>("nt_bigcode", ar, stride, steps, fit);
        run<16, 2>("sc1_vaddr", ar, stride, steps, fit);
        run<-1, 2>("nt_vaddr", ar, stride, steps, fit);
    }
    CK(hipFree(slab));
    return 0;
}
