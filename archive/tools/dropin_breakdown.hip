// tools/dropin_breakdown.hip -- where the per-call drop-in galois_w08_region_multiply
// spends its time on the host (not product).  Averages over many calls, one thread:
//   attr      hipPointerGetAttributes on pageable (malloc) memory, as device_view() does
//   getdev    hipGetDevice
//   enqueue   cec_region_multiply of 4 KiB device buffers: host time of the call alone
//             (no wait; the stream is drained every 64 calls outside the timing)
//   empty     an empty kernel launch: host time of the call alone
//   bigarg    the same with a 424-B by-value argument (CombineArgs' size)
//   capturing hipStreamIsCapturing on a plain stream
//   devcount  hipGetDeviceCount;  lasterr  hipGetLastError
//   arg64     a launch with a 64-B by-value argument (the two-slot arguments' size)
//   dev_call  galois_w08_region_multiply on device pointers, 4 KiB (launch + wait)
//   pageable  galois_w08_region_multiply on malloc'd buffers, 64 B and 4 KiB
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "cocytus_ec.h"
#include "galois.h"

__global__ void empty_kernel() {}
struct BigArgs {  // the size of the library's CombineArgs (48 stream bases + fields)
    void *p[53];
};
__global__ void bigarg_kernel(BigArgs a) { (void)a; }
struct SmallArgs {
    void *p[8];
};
__global__ void arg64_kernel(SmallArgs a) { (void)a; }

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0, int n) {
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main() {
    const int N = 20000;
    CK(hipSetDevice(0));
    char *h = static_cast<char *>(malloc(1 << 16)), *h2 = static_cast<char *>(malloc(1 << 16));
    memset(h, 7, 1 << 16);
    memset(h2, 9, 1 << 16);
    void *d1, *d2;
    CK(hipMalloc(&d1, 1 << 16));
    CK(hipMalloc(&d2, 1 << 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int i = 0; i < 200; ++i) galois_w08_region_multiply(h, 3, 4096, h2, 1);  // warm-up

    hipPointerAttribute_t at;
    auto t0 = clk::now();
    for (int i = 0; i < N; ++i) {
        if (hipPointerGetAttributes(&at, h + (i & 63)) != hipSuccess) (void)hipGetLastError();
    }
    const double attr = us_since(t0, N);

    int dev = 0;
    t0 = clk::now();
    for (int i = 0; i < N; ++i) (void)hipGetDevice(&dev);
    const double getdev = us_since(t0, N);

    int cnt = 0;
    t0 = clk::now();
    for (int i = 0; i < N; ++i) (void)hipGetDeviceCount(&cnt);
    const double devcount = us_since(t0, N);
    t0 = clk::now();
    for (int i = 0; i < N; ++i) (void)hipGetLastError();
    const double lasterr = us_since(t0, N);

    hipStreamCaptureStatus cs;
    t0 = clk::now();
    for (int i = 0; i < N; ++i) (void)hipStreamIsCapturing(s, &cs);
    const double capt = us_since(t0, N);

    double enq = 0, emp = 0, big = 0, a64 = 0;
    BigArgs ba{};
    SmallArgs sa{};
    for (int r = 0; r < N / 64; ++r) {
        auto t1 = clk::now();
        for (int i = 0; i < 64; ++i) cec_region_multiply(d1, 3, 4096, d2, 1, s);
        enq += std::chrono::duration<double, std::micro>(clk::now() - t1).count();
        CK(hipStreamSynchronize(s));
        t1 = clk::now();
        for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        emp += std::chrono::duration<double, std::micro>(clk::now() - t1).count();
        CK(hipStreamSynchronize(s));
        t1 = clk::now();
        for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(bigarg_kernel, dim3(1), dim3(64), 0, s, ba);
        big += std::chrono::duration<double, std::micro>(clk::now() - t1).count();
        CK(hipStreamSynchronize(s));
        t1 = clk::now();
        for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(arg64_kernel, dim3(4), dim3(64), 0, s, sa);
        a64 += std::chrono::duration<double, std::micro>(clk::now() - t1).count();
        CK(hipStreamSynchronize(s));
    }
    enq /= (N / 64) * 64;
    emp /= (N / 64) * 64;
    big /= (N / 64) * 64;
    a64 /= (N / 64) * 64;

    t0 = clk::now();
    for (int i = 0; i < N / 4; ++i)
        galois_w08_region_multiply(static_cast<char *>(d1), 3, 4096, static_cast<char *>(d2), 1);
    const double devcall = us_since(t0, N / 4);

    double pg[2];
    const int sizes[2] = {64, 4096};
    for (int z = 0; z < 2; ++z) {
        t0 = clk::now();
        for (int i = 0; i < N / 4; ++i) galois_w08_region_multiply(h, 3, sizes[z], h2, 1);
        pg[z] = us_since(t0, N / 4);
    }
    printf("{\"attr_us\": %.3f, \"getdev_us\": %.3f, \"devcount_us\": %.3f, \"lasterr_us\": %.3f, "
           "\"capturing_us\": %.3f, \"enqueue_us\": %.3f, \"empty_launch_us\": %.3f, "
           "\"arg64_launch_us\": %.3f, \"bigarg_launch_us\": %.3f, \"dev_call_4k_us\": %.2f, "
           "\"pageable_64_us\": %.2f, \"pageable_4k_us\": %.2f}\n",
           attr, getdev, devcount, lasterr, capt, enq, emp, a64, big, devcall, pg[0], pg[1]);
    return 0;
}
