// tools/delay_probe.hip -- why does the LDS engine's fixed-mask decode (D1 led by P1: two
// product rows staged per workgroup) run 5 % faster than the same kernel on an XOR-only
// mask (D0 led by P0: no staging), and than the PERM engine on either?  (not product)
//
// Bare XOR streams with the library's shape (64-lane workgroups, 1 KiB per workgroup and
// stream, nt loads and stores, arenas at the odd-4 KiB stride), 3 reads : 1 write (the
// decode) and 3 : 2 (the encode), with what the LDS engine adds between a wave's loads
// and its stores, one piece at a time:
//   plain      loads -> XOR -> stores
//   sleep2/8   s_sleep 2 / 8 (x 64 clocks) after the XOR
//   barrier    a workgroup barrier after the XOR
//   ldsrt      the XOR result through LDS (ds_write, barrier, ds_read) before the store
//   stage      the LDS engine's staging: a 512-B table read from L2 before the stream
//              loads, written to LDS, barrier; one LDS byte folded into the result
// Prints the median launch time per variant and shape, arena size from argv[1] (MiB).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/delay_probe.hip -o tools/delay_probe.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t ck_ = (x);                                              \
        if (ck_ != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(ck_));       \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GL __attribute__((address_space(1)))

struct Args {
    const uint8_t *r[3];
    uint8_t *w[2];
    const uint4 *table;  // 512 B (the "stage" variant)
};

enum { kPlain = 0, kSleep2, kSleep8, kBarrier, kLdsRt, kStage };

template <int W, int V>
__global__ __launch_bounds__(64) void k_stream(Args a) {
    __shared__ uint4 lds[64];
    const uint32_t off = blockIdx.x * 1024u + threadIdx.x * 16u;
    uint4 row = make_uint4(0, 0, 0, 0);
    if constexpr (V == kStage)
        if (threadIdx.x < 32) row = a.table[threadIdx.x];
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 3; ++i) acc ^= __builtin_nontemporal_load((const GL u32x4 *)((uintptr_t)a.r[i] + off));
    if constexpr (V == kStage) {
        if (threadIdx.x < 32) lds[threadIdx.x] = row;
        __syncthreads();
        acc.x ^= reinterpret_cast<const uint8_t *>(lds)[(acc.y & 511u)] & 0u;  // a dependent LDS read
        acc.y ^= reinterpret_cast<const uint8_t *>(lds)[(acc.z & 511u)];
    } else if constexpr (V == kSleep2) {
        __builtin_amdgcn_s_sleep(2);
    } else if constexpr (V == kSleep8) {
        __builtin_amdgcn_s_sleep(8);
    } else if constexpr (V == kBarrier) {
        __syncthreads();
    } else if constexpr (V == kLdsRt) {
        lds[threadIdx.x] = make_uint4(acc.x, acc.y, acc.z, acc.w);
        __syncthreads();
        const uint4 b = lds[threadIdx.x ^ 1];
        acc = u32x4{b.x, b.y, b.z, b.w};
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
        u32x4 v = acc;
        v.x ^= j;
        __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)a.w[j] + off));
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

template <int W, int V>
static float time_one(const Args &a, uint32_t grid) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    k_stream<W, V><<<grid, 64>>>(a);
    CK(hipEventRecord(e0, 0));
    const int iters = 10;
    for (int i = 0; i < iters; ++i) k_stream<W, V><<<grid, 64>>>(a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return t / iters;
}

int main(int argc, char **argv) {
    const uint64_t len = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 1024ull) << 20;
    uint64_t pages = (len + 4095) / 4096;
    if (pages % 2 == 0) ++pages;
    const uint64_t stride = pages * 4096;
    uint8_t *slab;
    CK(hipMalloc(&slab, 6 * stride));
    uint8_t *ar[6];
    for (int i = 0; i < 6; ++i) {
        ar[i] = slab + i * stride;
        k_fill<<<4096, 256>>>((uint64_t *)ar[i], len / 8, 0xC0C70000ull + i);
    }
    uint4 *table;
    CK(hipMalloc(&table, 512));
    CK(hipMemset(table, 0x5A, 512));
    CK(hipDeviceSynchronize());
    Args dec{{ar[1], ar[2], ar[4]}, {ar[5], ar[5]}, table};  // D0 rebuilt from D1, D2, P1
    Args enc{{ar[0], ar[1], ar[2]}, {ar[3], ar[4]}, table};
    const uint32_t grid = static_cast<uint32_t>(len / 1024);
    const char *names[] = {"plain", "sleep2", "sleep8", "barrier", "ldsrt", "stage"};
    const int rounds = 7;
    std::vector<float> t[2][6];
    for (int r = 0; r < rounds; ++r) {
        t[0][0].push_back(time_one<1, kPlain>(dec, grid));
        t[0][1].push_back(time_one<1, kSleep2>(dec, grid));
        t[0][2].push_back(time_one<1, kSleep8>(dec, grid));
        t[0][3].push_back(time_one<1, kBarrier>(dec, grid));
        t[0][4].push_back(time_one<1, kLdsRt>(dec, grid));
        t[0][5].push_back(time_one<1, kStage>(dec, grid));
        t[1][0].push_back(time_one<2, kPlain>(enc, grid));
        t[1][1].push_back(time_one<2, kSleep2>(enc, grid));
        t[1][2].push_back(time_one<2, kSleep8>(enc, grid));
        t[1][3].push_back(time_one<2, kBarrier>(enc, grid));
        t[1][4].push_back(time_one<2, kLdsRt>(enc, grid));
        t[1][5].push_back(time_one<2, kStage>(enc, grid));
    }
    for (int s = 0; s < 2; ++s)
        for (int v = 0; v < 6; ++v) {
            std::sort(t[s][v].begin(), t[s][v].end());
            const double ms = t[s][v][rounds / 2], bytes = (s ? 5.0 : 4.0) * len;
            printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"arena_MiB\": %llu, \"median_ms\": %.4f, "
                   "\"GBps\": %.0f, \"best_ms\": %.4f}\n",
                   s ? "3:2 encode" : "3:1 decode", names[v], (unsigned long long)(len >> 20), ms,
                   bytes / (ms * 1e6), t[s][v][0]);
        }
    CK(hipFree(table));
    CK(hipFree(slab));
    return 0;
}
