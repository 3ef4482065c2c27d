/*
 * tools/dropin_latency.c -- per-call cost of the drop-in galois_w08_region_multiply as
 * the unchanged server calls it (one synchronous call per SET / per parity apply /
 * per recovery unit), on pageable host buffers, for several region sizes.
 *   gcc -O2 -Iinclude tools/dropin_latency.c -Lcocytus_amd -lJerasure \
 *       -Wl,-rpath,$PWD/cocytus_amd -o tools/dropin_latency.bin
 */
#include <galois.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(void) {
    const int sizes[] = {64, 4098, 65536, 1 << 20};
    char *a = malloc(1 << 20), *b = malloc(1 << 20);
    for (int i = 0; i < (1 << 20); ++i) { a[i] = (char)(i * 7); b[i] = (char)(i * 13); }
    galois_w08_region_multiply(a, 245, 4096, b, 1);  /* warm up: device, stream, staging */
    for (int s = 0; s < 4; ++s) {
        const int n = sizes[s], iters = n >= (1 << 20) ? 200 : 2000;
        const double t0 = now();
        for (int i = 0; i < iters; ++i) galois_w08_region_multiply(a, 245, n, b, 1);
        const double t = (now() - t0) / iters;
        printf("{\"bytes\": %d, \"us_per_call\": %.2f, \"GBps\": %.3f}\n", n, t * 1e6, n / t / 1e9);
    }
    return 0;
}
