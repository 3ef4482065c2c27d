/*
 * tests/dropin/dropin_threads.c -- re-entrancy of the drop-in symbols: T pthreads call
 * galois_w08_region_multiply concurrently (each on its own buffers, mixed sizes, odd
 * alignments, all four argument forms), and each thread checks its own results with a
 * private scalar GF(2^8) (poly 0x11D) written here.  Exit status 0 = all equal.
 *   gcc -O1 -Iinclude tests/dropin/dropin_threads.c -Lcocytus_amd -lJerasure -lpthread
 */
#include <galois.h>

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int gmul(int a, int b) {
    int r = 0;
    while (b) {
        if (b & 1) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x100) a ^= 0x11D;
    }
    return r;
}

typedef struct {
    int id, iters, bad;
} arg_t;

static uint64_t next(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void *worker(void *p) {
    arg_t *a = (arg_t *)p;
    uint64_t s = 0xC0C70000ull + (uint64_t)a->id;
    unsigned char *src = malloc(300000 + 64), *dst = malloc(300000 + 64), *exp = malloc(300000 + 64);
    for (int it = 0; it < a->iters; ++it) {
        const int n = (int)(next(&s) % (it % 4 == 3 ? 300000 : 5000)) + 1;
        const int so = (int)(next(&s) % 17), dso = (int)(next(&s) % 17);
        const int c = (int)(next(&s) % 256), form = it % 4;
        for (int i = 0; i < n + 32; ++i) {
            src[i] = (unsigned char)next(&s);
            dst[i] = (unsigned char)next(&s);
        }
        memcpy(exp, dst, n + 32);
        if (form == 0) {            /* r2 ^= c * region (every Cocytus call site) */
            for (int i = 0; i < n; ++i) exp[dso + i] ^= (unsigned char)gmul(c, src[so + i]);
            galois_w08_region_multiply((char *)src + so, c, n, (char *)dst + dso, 1);
        } else if (form == 1) {     /* r2 = c * region */
            for (int i = 0; i < n; ++i) exp[dso + i] = (unsigned char)gmul(c, src[so + i]);
            galois_w08_region_multiply((char *)src + so, c, n, (char *)dst + dso, 0);
        } else if (form == 2) {     /* in place: region = c * region */
            for (int i = 0; i < n; ++i) exp[dso + i] = (unsigned char)gmul(c, exp[dso + i]);
            galois_w08_region_multiply((char *)dst + dso, c, n, NULL, 0);
        } else {                    /* the diff form: multby 1 (memcached.c:2681) */
            for (int i = 0; i < n; ++i) exp[dso + i] ^= src[so + i];
            galois_w08_region_multiply((char *)src + so, 1, n, (char *)dst + dso, 1);
        }
        if (memcmp(dst, exp, n + 32) != 0) {
            fprintf(stderr, "thread %d iter %d: mismatch (n=%d c=%d form=%d)\n", a->id, it, n, c, form);
            a->bad++;
        }
    }
    free(src);
    free(dst);
    free(exp);
    return NULL;
}

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 8, iters = argc > 2 ? atoi(argv[2]) : 200;
    pthread_t th[64];
    arg_t args[64];
    for (int t = 0; t < T; ++t) {
        args[t].id = t;
        args[t].iters = iters;
        args[t].bad = 0;
        pthread_create(&th[t], NULL, worker, &args[t]);
    }
    int bad = 0;
    for (int t = 0; t < T; ++t) {
        pthread_join(th[t], NULL);
        bad += args[t].bad;
    }
    printf("dropin threads: %d x %d calls, %d mismatches\n", T, iters, bad);
    return bad ? 1 : 0;
}
