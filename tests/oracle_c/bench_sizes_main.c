/* tests/oracle_c/bench_sizes_main.c -- the CPU-baseline leg's thread split (uniform and
 * mixed value sizes, more threads than stripes) under ASan + UBSan: see
 * tests/test_dist_harness.py::test_cpu_baseline_split_under_asan. */
#include <stdio.h>
int ref_bench_encode_decode_sizes(int k, int m, long n, const long *lens, long nstripes, int threads,
                                  int reps, int do_decode, int samples, double *t);
int ref_bench_encode_decode_samples(int k, int m, long n, long nstripes, int threads,
                                    int reps, int do_decode, int samples, double *t);
int main(void) {
    long lens[7] = {256, 1000, 4096, 70000, 17, 300000, 4098};
    double t[2];
    int threads[] = {1, 3, 64};
    for (int i = 0; i < 3; ++i) {
        if (ref_bench_encode_decode_sizes(3, 2, 0, lens, 7, threads[i], 1, 1, 2, t)) return 1;
        if (ref_bench_encode_decode_samples(4, 2, 65536, 5, threads[i], 1, 1, 2, t)) return 1;
    }
    puts("ok");
    return 0;
}
