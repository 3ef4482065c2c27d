// tools/launch_latency.hip -- floor of one synchronous GPU call from the host (not product):
// what bounds the per-call drop-in galois_w08_region_multiply.
//   A  empty kernel + hipStreamSynchronize
//   B  empty kernel that then sets a flag in mapped pinned memory; host spins on the flag
//   C  64-B kernel reading / writing mapped pinned memory + hipStreamSynchronize
//   D  the same + host spin on a completion flag written by the kernel
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

__global__ void k_empty() {}
__global__ void k_flag(volatile unsigned *flag, unsigned v) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        *flag = v;
    }
}
__global__ void k_xor(const unsigned char *src, unsigned char *dst, int n, volatile unsigned *flag, unsigned v) {
    const int i = threadIdx.x;
    if (i < n) dst[i] ^= src[i];
    if (flag) {
        __syncthreads();
        if (i == 0) {
            __threadfence_system();
            *flag = v;
        }
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *flag;
    unsigned char *buf;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&buf, 8192, hipHostMallocMapped | hipHostMallocCoherent));
    unsigned *dflag;
    unsigned char *dbuf;
    CK(hipHostGetDevicePointer((void **)&dflag, flag, 0));
    CK(hipHostGetDevicePointer((void **)&dbuf, buf, 0));
    *flag = 0;
    const int iters = 2000;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [&](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count() / iters; };
    for (int warm = 0; warm < 2; ++warm) {
        auto t0 = now();
        for (int i = 0; i < iters; ++i) {
            hipLaunchKernelGGL(k_empty, 1, 64, 0, s);
            CK(hipStreamSynchronize(s));
        }
        auto t1 = now();
        for (int i = 0; i < iters; ++i) {
            const unsigned v = 1000000u * warm + i + 1;
            hipLaunchKernelGGL(k_flag, 1, 64, 0, s, (volatile unsigned *)dflag, v);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
            }
        }
        CK(hipStreamSynchronize(s));
        auto t2 = now();
        for (int i = 0; i < iters; ++i) {
            hipLaunchKernelGGL(k_xor, 1, 64, 0, s, (const unsigned char *)dbuf, dbuf + 4096, 64,
                               (volatile unsigned *)nullptr, 0u);
            CK(hipStreamSynchronize(s));
        }
        auto t3 = now();
        for (int i = 0; i < iters; ++i) {
            const unsigned v = 2000000u + 1000000u * warm + i + 1;
            hipLaunchKernelGGL(k_xor, 1, 64, 0, s, (const unsigned char *)dbuf, dbuf + 4096, 64,
                               (volatile unsigned *)dflag, v);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
            }
        }
        CK(hipStreamSynchronize(s));
        auto t4 = now();
        if (warm)
            printf("A empty+sync %.2f us | B empty+flag spin %.2f us | C 64B mapped+sync %.2f us | "
                   "D 64B mapped+flag spin %.2f us\n",
                   us(t0, t1), us(t1, t2), us(t2, t3), us(t3, t4));
    }
    return 0;
}
