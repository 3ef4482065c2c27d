// tools/stream_probe.hip -- what the HIP runtime does with the handle of a destroyed
// stream (hipStreamSynchronize / hipStreamQuery / hipEventRecord on it): the
// libcocytus_ec trackers rely on it failing cleanly (not product).
#include <hip/hip_runtime.h>

#include <cstdio>

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    (void)hipStreamSynchronize(s);
    if (hipStreamDestroy(s) != hipSuccess) return 1;
    hipError_t a = hipStreamSynchronize(s);
    printf("hipStreamSynchronize(destroyed) = %d (%s)\n", (int)a, hipGetErrorString(a));
    (void)hipGetLastError();
    hipError_t b = hipStreamQuery(s);
    printf("hipStreamQuery(destroyed) = %d (%s)\n", (int)b, hipGetErrorString(b));
    (void)hipGetLastError();
    hipEvent_t e;
    (void)hipEventCreate(&e);
    hipError_t c = hipEventRecord(e, s);
    printf("hipEventRecord(destroyed) = %d (%s)\n", (int)c, hipGetErrorString(c));
    fflush(stdout);
    return 0;
}
