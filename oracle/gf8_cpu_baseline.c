/*
 * oracle/gf8_cpu_baseline.c -- the timed CPU baseline (bench.py cpu_baseline leg).
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY; never linked into the product.
 *
 * The reference CPU path is Jerasure + GF-Complete, absent from this image
 * (SURVEY.md §8c), so this is the "restated CPU baseline": GF-Complete's default
 * w=8 region multiply (SPLIT 8,4: two 16-entry product tables per coefficient,
 * one per nibble, looked up with pshufb) restated with 32-byte AVX2 vpshufb, and
 * chained exactly like the reference's call sites:
 *   encode  = K SETs into zero parity, one region multiply per (parity, shard)
 *             (memcached.c:2681 + 7764 with old = 0);
 *   decode  = residual build per survivor (recovery.c:79-93) + leader solve
 *             (memcached.c:7913-7922) into a zeroed buffer.
 */
#include "gf8_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#define HAVE_X86 1
#endif

int ref_simd_available(void)
{
#if HAVE_X86
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") ? 1 : 0;
#else
    return 0;
#endif
}

#if HAVE_X86
__attribute__((target("avx2")))
static void region_mul_xor_avx2(const uint8_t *src, int c, long n, uint8_t *dst)
{
    uint8_t lo[16], hi[16];
    for (int i = 0; i < 16; ++i) {
        lo[i] = (uint8_t)ref_gf_mul(c, i);
        hi[i] = (uint8_t)ref_gf_mul(c, i << 4);
    }
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    const __m256i mask = _mm256_set1_epi8(0x0F);
    long i = 0;
    if (c == 1) {
        for (; i + 32 <= n; i += 32) {
            __m256i s = _mm256_loadu_si256((const __m256i *)(src + i));
            __m256i d = _mm256_loadu_si256((const __m256i *)(dst + i));
            _mm256_storeu_si256((__m256i *)(dst + i), _mm256_xor_si256(s, d));
        }
    } else {
        for (; i + 32 <= n; i += 32) {
            __m256i s = _mm256_loadu_si256((const __m256i *)(src + i));
            __m256i d = _mm256_loadu_si256((const __m256i *)(dst + i));
            __m256i l = _mm256_shuffle_epi8(tlo, _mm256_and_si256(s, mask));
            __m256i h = _mm256_shuffle_epi8(thi, _mm256_and_si256(_mm256_srli_epi64(s, 4), mask));
            d = _mm256_xor_si256(d, _mm256_xor_si256(l, h));
            _mm256_storeu_si256((__m256i *)(dst + i), d);
        }
    }
    for (; i < n; ++i) dst[i] ^= (uint8_t)(lo[src[i] & 15] ^ hi[src[i] >> 4]);
}
#endif

void ref_region_multiply_simd(const uint8_t *region, int multby, long nbytes, uint8_t *r2)
{
    if (multby == 0 || nbytes <= 0) return;
#if HAVE_X86
    if (ref_simd_available()) { region_mul_xor_avx2(region, multby, nbytes, r2); return; }
#endif
    ref_region_multiply((uint8_t *)region, multby, nbytes, r2, 1);
}

typedef struct {
    const int *matrix;
    int k, m, do_decode, reps, samples;
    long n, s0, s1;
    const long *offs, *lens; /* per-stripe offset / length (mixed sizes), or NULL: s * n, n */
    uint8_t **data, **parity, *out, *res;
    pthread_barrier_t *bar;
} bench_arg;

/* splitmix64 bytes [lo, hi) of the stream seeded `seed` (8-byte words; word w is
 * the w+1-th output), the synthetic input of SURVEY §8d. */
static void fill_splitmix(uint8_t *buf, uint64_t seed, size_t lo, size_t hi)
{
    for (size_t i = lo & ~(size_t)7; i < hi; i += 8) {
        uint64_t z = seed + (uint64_t)(i / 8 + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (i >= lo && i + 8 <= hi) {
            memcpy(buf + i, &z, 8);
            continue;
        }
        for (int b = 0; b < 8; ++b)
            if (i + (size_t)b >= lo && i + (size_t)b < hi) buf[i + (size_t)b] = (uint8_t)(z >> (8 * b));
    }
}

static void *bench_worker(void *p)
{
    bench_arg *a = (bench_arg *)p;
    const int k = a->k, m = a->m;
    /* each thread fills and first-touches its own stripes (NUMA-local pages on a
     * multi-socket host); untimed */
    const int none = a->s1 <= a->s0; /* more threads than stripes: nothing to fill */
    const size_t lo = none ? 0 : a->offs ? (size_t)a->offs[a->s0] : (size_t)a->s0 * (size_t)a->n;
    const size_t hi = none ? 0
                      : a->offs ? (size_t)(a->offs[a->s1 - 1] + a->lens[a->s1 - 1])
                                : (size_t)a->s1 * (size_t)a->n;
    for (int j = 0; j < k; ++j) fill_splitmix(a->data[j], 0xC0C70001ull + (uint64_t)j, lo, hi);
    for (int q = 0; q < m; ++q) memset(a->parity[q] + lo, 0, hi - lo);
    pthread_barrier_wait(a->bar);
    for (int smp = 0; smp < a->samples; ++smp) {
    for (int r = 0; r < a->reps; ++r) {
        for (long s = a->s0; s < a->s1; ++s) {
            const long off = a->offs ? a->offs[s] : s * a->n, n = a->lens ? a->lens[s] : a->n;
            for (int q = 0; q < m; ++q) memset(a->parity[q] + off, 0, (size_t)n);
            for (int j = 0; j < k; ++j)
                for (int q = 0; q < m; ++q)
                    ref_region_multiply_simd(a->data[j] + off, a->matrix[(k + q) * k + j], n,
                                             a->parity[q] + off);
            if (!a->do_decode) continue;
            /* one lost data shard per stripe, leader parity rotates */
            const int lost = (int)(s % k), leader = k + (int)((s / k) % m);
            memcpy(a->res, a->parity[leader - k] + off, (size_t)n);
            for (int j = 0; j < k; ++j)
                if (j != lost)
                    ref_region_multiply_simd(a->data[j] + off, a->matrix[leader * k + j], n, a->res);
            const int inv = ref_gf_div(1, a->matrix[leader * k + lost]);
            memset(a->out, 0, (size_t)n);
            ref_region_multiply_simd(a->res, inv, n, a->out);
        }
    }
    pthread_barrier_wait(a->bar);  /* end of sample smp: the main thread timestamps it */
    }
    return NULL;
}

/* `samples` timed passes of `reps` repetitions each over the same filled stripes
 * (one fill, untimed); t[i] = seconds of sample i (CLOCK_MONOTONIC between the
 * barriers that end consecutive samples: every thread has finished it). */
/* lens != NULL: stripe s has lens[s] bytes (mixed sizes, SURVEY §8d cfg 3), packed at
 * 16-B aligned offsets (ecalloc.c:176); threads split the stripes by bytes; n is then
 * ignored.  lens == NULL: every stripe has n bytes. */
int ref_bench_encode_decode_sizes(int k, int m, long n, const long *lens, long nstripes, int threads,
                                  int reps, int do_decode, int samples, double *t)
{
    if (threads < 1) threads = 1;
    if (samples < 1 || !t || nstripes < 1) return -1;
    int *matrix = ref_big_vandermonde(k + m, k);
    uint8_t *data[32], *parity[32];
    long *offs = NULL;
    size_t bytes = (size_t)n * (size_t)nstripes;
    long maxlen = n;
    if (lens) {
        offs = (long *)malloc(sizeof(long) * (size_t)nstripes);
        long o = 0;
        maxlen = 0;
        for (long s = 0; s < nstripes; ++s) {
            offs[s] = o;
            o = (o + lens[s] + 15) & ~15L;
            if (lens[s] > maxlen) maxlen = lens[s];
        }
        bytes = (size_t)o;
    }
    /* filled by the workers, each its own stripes (bench_worker) */
    for (int j = 0; j < k; ++j) data[j] = (uint8_t *)aligned_alloc(64, (bytes + 63) & ~(size_t)63);
    for (int q = 0; q < m; ++q) parity[q] = (uint8_t *)aligned_alloc(64, (bytes + 63) & ~(size_t)63);
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    bench_arg *args = (bench_arg *)calloc((size_t)threads, sizeof(bench_arg));
    for (int th = 0; th < threads; ++th) {
        bench_arg *a = &args[th];
        a->matrix = matrix; a->k = k; a->m = m; a->n = n; a->reps = reps; a->do_decode = do_decode;
        a->samples = samples;
        a->offs = offs; a->lens = lens;
        if (lens) { /* by bytes: the first stripe starting at or past th / threads of them */
            long lo = 0, hi = 0;
            while (lo < nstripes && (size_t)offs[lo] * (size_t)threads < bytes * (size_t)th) ++lo;
            hi = lo;
            while (hi < nstripes && (size_t)offs[hi] * (size_t)threads < bytes * (size_t)(th + 1)) ++hi;
            a->s0 = lo;
            a->s1 = th + 1 == threads ? nstripes : hi;
        } else {
            a->s0 = nstripes * th / threads;
            a->s1 = nstripes * (th + 1) / threads;
        }
        a->data = data; a->parity = parity; a->bar = &bar;
        a->out = (uint8_t *)aligned_alloc(64, ((size_t)maxlen + 63) & ~(size_t)63);
        a->res = (uint8_t *)aligned_alloc(64, ((size_t)maxlen + 63) & ~(size_t)63);
        pthread_create(&tid[th], NULL, bench_worker, a);
    }
    struct timespec t0, t1;
    pthread_barrier_wait(&bar);  /* every worker has filled its stripes */
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int smp = 0; smp < samples; ++smp) {
        pthread_barrier_wait(&bar);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        t[smp] = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        t0 = t1;
    }
    for (int th = 0; th < threads; ++th) pthread_join(tid[th], NULL);
    for (int th = 0; th < threads; ++th) { free(args[th].out); free(args[th].res); }
    for (int j = 0; j < k; ++j) free(data[j]);
    for (int q = 0; q < m; ++q) free(parity[q]);
    free(args); free(tid); free(matrix); free(offs);
    pthread_barrier_destroy(&bar);
    return 0;
}

int ref_bench_encode_decode_samples(int k, int m, long n, long nstripes, int threads,
                                    int reps, int do_decode, int samples, double *t)
{
    return ref_bench_encode_decode_sizes(k, m, n, NULL, nstripes, threads, reps, do_decode, samples, t);
}

double ref_bench_encode_decode(int k, int m, long n, long nstripes, int threads,
                               int reps, int do_decode)
{
    double t = 0.0;
    ref_bench_encode_decode_samples(k, m, n, nstripes, threads, reps, do_decode, 1, &t);
    return t;
}

double ref_bench_recover(const uint8_t *parity, const uint8_t *const *peers, const int *coefs,
                         int npeers, int inv, long nbuf, uint8_t *residual, uint8_t *out)
{
    const long unit = 4096;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int p = 0; p < npeers; ++p)
        for (long u = 0; u < nbuf; u += unit) {
            const long len = nbuf - u < unit ? nbuf - u : unit;
            if (p == 0) memcpy(residual + u, parity + u, (size_t)len);
            ref_region_multiply_simd(peers[p] + u, coefs[p], len, residual + u);
        }
    memset(out, 0, (size_t)nbuf);
    ref_region_multiply_simd(residual, inv, nbuf, out);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

double ref_bench_apply(const uint8_t *stage, const uint64_t *soffs, const uint64_t *addrs,
                       const uint32_t *lens, const int *coefs, int n, uint8_t *parity)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < n; ++i)
        ref_region_multiply_simd(stage + soffs[i], coefs[i], (long)lens[i], parity + addrs[i]);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

static double secs(struct timespec a, struct timespec b)
{
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

double ref_bench_set_diffs(const uint8_t *values, const uint64_t *voffs, const uint8_t *ecmem,
                           const uint64_t *addrs, const uint32_t *lens, int n, uint8_t *diffs,
                           const uint64_t *doffs)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < n; ++i) { /* memcached.c:2678-2681 */
        memcpy(diffs + doffs[i], values + voffs[i], lens[i]);
        ref_region_multiply_simd(ecmem + addrs[i], 1, (long)lens[i], diffs + doffs[i]);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return secs(t0, t1);
}

double ref_bench_recover_requests(const uint8_t *ecmem, const int *starts, int nreq, int units,
                                  const uint8_t *const *replies, int npeers, const int *coefs, int inv,
                                  uint8_t *const *outs)
{
    const size_t U = 4096, nbuf = (size_t)units * U;
    uint8_t **unit = (uint8_t **)calloc((size_t)nreq * (size_t)units, sizeof(uint8_t *));
    uint8_t **data = (uint8_t **)calloc((size_t)nreq, sizeof(uint8_t *));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int q = 0; q < nreq; ++q)
        for (int p = 0; p < npeers; ++p)
            for (int i = 0; i < units; ++i) { /* recovery.c:72-94 */
                uint8_t **u = &unit[(size_t)q * (size_t)units + (size_t)i];
                if (!*u) { /* first touch: malloc(UNITSIZE) + memcpy of the parity unit */
                    *u = (uint8_t *)malloc(U);
                    memcpy(*u, ecmem + ((size_t)starts[q] + (size_t)i) * U, U);
                }
                ref_region_multiply_simd(replies[(size_t)q * (size_t)npeers + (size_t)p] + (size_t)i * U, coefs[p],
                                         (long)U, *u);
            }
    for (int q = 0; q < nreq; ++q) { /* memcached.c:7853-7922, one lost shard */
        uint8_t *buf = (uint8_t *)malloc(nbuf);
        for (int i = 0; i < units; ++i) memcpy(buf + (size_t)i * U, unit[(size_t)q * (size_t)units + (size_t)i], U);
        data[q] = (uint8_t *)calloc(1, nbuf);
        ref_region_multiply_simd(buf, inv, (long)nbuf, data[q]);
        free(buf);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (int q = 0; q < nreq; ++q) {
        memcpy(outs[q], data[q], nbuf);
        free(data[q]);
    }
    for (size_t x = 0; x < (size_t)nreq * (size_t)units; ++x) free(unit[x]);
    free(unit);
    free(data);
    return secs(t0, t1);
}
