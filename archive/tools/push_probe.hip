// tools/push_probe.hip -- can the host PUSH a drop-in request into device memory, and
// does that beat the resident worker's pull over PCIe?
//
// Modes (one resident workgroup each, 4 KiB requests, ping-pong from the host):
//   pull : mailbox + operands in mapped pinned host memory; the worker polls and reads
//          them over PCIe (the resident worker of commit 3200187, since removed)
//   push : mailbox + operands in fine-grained device memory that the host writes through
//          its mapping; the worker polls and reads HBM, writes the result and the
//          acknowledgement into mapped pinned host memory
// Prints one line per mode: us per request (host post -> host sees the result).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ inline void ld128(const void *p, u32x4 &v) {
    __asm__ volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
}
__device__ inline void st128(void *p, const u32x4 &v) {
    __asm__ volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ inline void wait(u32x4 &v) { __asm__ volatile("s_waitcnt vmcnt(0)" : "+v"(v) : : "memory"); }
__device__ inline void drain() { __asm__ volatile("s_waitcnt vmcnt(0)" : : : "memory"); }

// req: [0] seq, [1] stop; in: 4 KiB operand; out: 4 KiB result (host); ack: [0] done
__global__ __launch_bounds__(256) void worker(const uint32_t *req, const uint8_t *in, uint8_t *out, uint32_t *ack,
                                              uint64_t life) {
    __shared__ uint32_t go, seq_s;
    const uint64_t t0 = wall_clock64();
    uint32_t last = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t g = 0;
            for (;;) {
                if (wall_clock64() - t0 > life) break;
                const uint64_t w = __hip_atomic_load(reinterpret_cast<const uint64_t *>(req), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM);
                if (static_cast<uint32_t>(w) != last) {
                    g = 1;
                    seq_s = static_cast<uint32_t>(w);
                    break;
                }
                if (w >> 32) break;
                __builtin_amdgcn_s_sleep(1);
            }
            go = g;
        }
        __syncthreads();
        if (!go) break;
        const uint32_t seq = seq_s;
        u32x4 x;
        ld128(in + threadIdx.x * 16, x);
        wait(x);
        x ^= u32x4{seq, seq, seq, seq};
        st128(out + threadIdx.x * 16, x);
        drain();
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(ack, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = seq;
        }
        __syncthreads();
    }
}

static double run(const char *name, uint32_t *req_h, const uint32_t *req_d, uint8_t *in_h, const uint8_t *in_d,
                  uint8_t *out_h, uint8_t *out_d, uint32_t *ack_h, uint32_t *ack_d, int iters) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    __atomic_store_n(&req_h[1], 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&req_h[0], 0u, __ATOMIC_RELEASE);
    __atomic_store_n(ack_h, 0u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(worker, dim3(1), dim3(256), 0, s, req_d, in_d, out_d, ack_d, uint64_t(khz) * 1000 * 20);
    CK(hipGetLastError());
    static uint8_t src[4096];
    int bad = 0;
    double best = 1e9, sum = 0;
    for (int i = 1; i <= iters; ++i) {
        for (int b = 0; b < 4096; b += 64) src[b] = static_cast<uint8_t>(i + b);
        const auto t0 = std::chrono::steady_clock::now();
        memcpy(in_h, src, 4096);
        __atomic_store_n(&req_h[0], static_cast<uint32_t>(i), __ATOMIC_RELEASE);
        const auto tl = t0 + std::chrono::seconds(5);
        while (__atomic_load_n(ack_h, __ATOMIC_ACQUIRE) != static_cast<uint32_t>(i)) {
            __builtin_ia32_pause();
            if (std::chrono::steady_clock::now() > tl) {
                fprintf(stderr, "%s: no reply\n", name);
                __atomic_store_n(&req_h[1], 1u, __ATOMIC_RELEASE);
                CK(hipStreamSynchronize(s));
                return -1;
            }
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        for (int b = 0; b < 4096; b += 64)
            if (out_h[b] != static_cast<uint8_t>(src[b] ^ (i & 0xFF))) ++bad;
        if (i > 100) {
            sum += us;
            if (us < best) best = us;
        }
    }
    __atomic_store_n(&req_h[1], 1u, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    printf("{\"mode\": \"%s\", \"us_per_request\": %.2f, \"best_us\": %.2f, \"mismatches\": %d}\n", name,
           sum / (iters - 100), best, bad);
    fflush(stdout);
    return sum / (iters - 100);
}

int main() {
    CK(hipSetDevice(0));
    const int iters = 5000;
    // result + acknowledgement always in mapped pinned host memory
    uint8_t *out_h;
    uint32_t *ack_h;
    CK(hipHostMalloc(reinterpret_cast<void **>(&out_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(reinterpret_cast<void **>(&ack_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    uint8_t *out_d;
    uint32_t *ack_d;
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&out_d), out_h, 0));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ack_d), ack_h, 0));
    {  // pull
        uint32_t *req_h;
        uint8_t *in_h;
        CK(hipHostMalloc(reinterpret_cast<void **>(&req_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostMalloc(reinterpret_cast<void **>(&in_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
        uint32_t *req_d;
        uint8_t *in_d;
        CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&req_d), req_h, 0));
        CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&in_d), in_h, 0));
        run("pull", req_h, req_d, in_h, in_d, out_h, out_d, ack_h, ack_d, iters);
    }
    {  // push: fine-grained device memory, written by the host through its mapping
        void *dev = nullptr;
        CK(hipExtMallocWithFlags(&dev, 8192, hipDeviceMallocFinegrained));
        hipPointerAttribute_t at;
        CK(hipPointerGetAttributes(&at, dev));
        printf("{\"finegrained_vram\": {\"type\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\"}}\n",
               static_cast<int>(at.type), at.hostPointer, at.devicePointer);
        fflush(stdout);
        uint8_t *hp = static_cast<uint8_t *>(at.hostPointer ? at.hostPointer : dev);
        // a host write that faults ends this probe here: the pull line above stands
        memset(hp, 0, 8192);
        run("push", reinterpret_cast<uint32_t *>(hp + 4096), reinterpret_cast<const uint32_t *>(
                static_cast<uint8_t *>(dev) + 4096), hp, static_cast<const uint8_t *>(dev), out_h, out_d, ack_h, ack_d,
            iters);
    }
    return 0;
}
