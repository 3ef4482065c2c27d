/*
 * tests/dropin/cache_threads.c -- the runtime's shared state under concurrent use:
 * T host threads, one stream each, every iteration a different RS(k,m) code (so the
 * coefficient-table cache, capped at a few entries, evicts while other threads launch),
 * a fresh plan per batch (the idle-buffer cache), encode, a random single-erasure decode,
 * destroy; plus region multiply by c then by 1/c, and now and then cec_cache_trim() from
 * one thread while the others run.  Every result is checked by a size-independent
 * property (rebuilt shard == original, c * (1/c) * x == x), no oracle needed.
 * Prints one JSON line; exit 0 iff every check passed.
 *   usage: cache_threads [THREADS [ITERS [PATTERN_LIMIT]]]
 */
#include <cocytus_ec.h>
#include <galois.h>
#include <reed_sol.h>

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { MAXK = 6, MAXM = 3, NSTRIPE = 48 };
static const size_t n = 4096;

typedef struct {
    int id, iters;
    long checks, bad, errors;
} targ;

static uint64_t next(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define TRY(x)                                                              \
    do {                                                                    \
        if ((x) < 0) {                                                      \
            fprintf(stderr, "thread %d: %s: %s\n", a->id, #x, cec_last_error()); \
            ++a->errors;                                                    \
            goto out;                                                       \
        }                                                                   \
    } while (0)

static void *worker(void *p) {
    targ *a = (targ *)p;
    const size_t L = n * NSTRIPE;
    uint64_t rng = 0xC0C70100ull + (uint64_t)a->id;
    void *stream = NULL, *slab = NULL;
    uint8_t *ar[MAXK + MAXM + MAXK];
    uint8_t *h = malloc(L), *g = malloc(L), *w = malloc(L);
    cec_extent ext[NSTRIPE];
    int *matrix = NULL;
    if (cec_set_device(0) < 0 || cec_stream_create(&stream) < 0) {
        ++a->errors;
        goto out;
    }
    TRY(cec_arenas_alloc(MAXK + MAXM + MAXK, L, ar, &slab));
    for (int j = 0; j < MAXK; ++j) {
        for (size_t i = 0; i < L; i += 8) {
            const uint64_t z = next(&rng);
            memcpy(h + i, &z, 8);
        }
        TRY(cec_copy(ar[j], h, L, stream));
        TRY(cec_stream_synchronize(stream));
    }
    for (int it = 0; it < a->iters; ++it) {
        const int k = 2 + (int)(next(&rng) % (MAXK - 1)), m = 1 + (int)(next(&rng) % MAXM);
        matrix = reed_sol_big_vandermonde_distribution_matrix(k + m, k, 8);
        if (!matrix) {
            ++a->errors;
            goto out;
        }
        uint8_t *data[MAXK], *parity[MAXM], *outv[MAXK];
        const uint8_t *arenas[MAXK + MAXM];
        for (int j = 0; j < k; ++j) {
            data[j] = ar[j];
            arenas[j] = ar[j];
        }
        for (int q = 0; q < m; ++q) parity[q] = ar[MAXK + q], arenas[k + q] = ar[MAXK + q];
        for (int j = 0; j < k; ++j) outv[j] = ar[MAXK + MAXM + j];
        for (int s = 0; s < NSTRIPE; ++s) {
            ext[s].off = (uint64_t)s * n;
            ext[s].src_off = 0;
            ext[s].len = (uint32_t)(n - (next(&rng) % 64));  /* ragged values too */
            ext[s].pattern = 0;
        }
        cec_plan *plan = NULL;
        TRY(cec_plan_create(&plan, ext, NSTRIPE, stream));
        TRY(cec_encode(k, m, matrix, (const uint8_t *const *)data, parity, plan, stream));
        const int lost = (int)(next(&rng) % (uint64_t)k), leader = k + (int)(next(&rng) % (uint64_t)m);
        int conn[MAXK + MAXM];
        for (int i = 0; i < k + m; ++i) conn[i] = i != lost;
        const uint32_t mask = cec_recovery_mask(k, m, leader, conn);
        TRY(cec_decode(k, m, matrix, &mask, 1, arenas, outv, plan, stream));
        TRY(cec_copy(g, outv[lost], L, stream));
        TRY(cec_copy(w, data[lost], L, stream));
        TRY(cec_stream_synchronize(stream));
        TRY(cec_plan_destroy(plan));
        for (int s = 0; s < NSTRIPE; ++s, ++a->checks)
            if (memcmp(g + (size_t)s * n, w + (size_t)s * n, ext[s].len) != 0) ++a->bad;
        /* c * x, then (1/c) * that == x, through the region multiply */
        const int c = 2 + (int)(next(&rng) % 254), ci = galois_single_divide(1, c, 8);
        uint8_t *x = ar[0], *y = ar[MAXK + MAXM], *z = ar[MAXK + MAXM + 1];
        TRY(cec_region_multiply(x, c, L, y, 0, stream));
        TRY(cec_region_multiply(y, ci, L, z, 0, stream));
        TRY(cec_copy(g, z, L, stream));
        TRY(cec_copy(w, x, L, stream));
        TRY(cec_stream_synchronize(stream));
        ++a->checks;
        if (memcmp(g, w, L) != 0) ++a->bad;
        if (a->id == 0 && it % 17 == 16) TRY(cec_cache_trim());  /* while the others launch */
        free(matrix);
        matrix = NULL;
    }
out:
    free(matrix);
    if (slab) cec_arenas_free(slab);
    if (stream) cec_stream_destroy(stream);
    free(h);
    free(g);
    free(w);
    return NULL;
}

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 8, iters = argc > 2 ? atoi(argv[2]) : 100;
    const int limit = argc > 3 ? atoi(argv[3]) : 6;
    if (cec_device_check() != CEC_OK || cec_cache_set_pattern_limit(limit) != CEC_OK) {
        fprintf(stderr, "%s\n", cec_last_error());
        return 1;
    }
    pthread_t tid[64];
    targ args[64];
    const int nt = T < 64 ? T : 64;
    for (int t = 0; t < nt; ++t) {
        memset(&args[t], 0, sizeof args[t]);
        args[t].id = t;
        args[t].iters = iters;
        pthread_create(&tid[t], NULL, worker, &args[t]);
    }
    long checks = 0, bad = 0, errors = 0;
    for (int t = 0; t < nt; ++t) {
        pthread_join(tid[t], NULL);
        checks += args[t].checks;
        bad += args[t].bad;
        errors += args[t].errors;
    }
    cec_cache_info ci;
    cec_cache_get_info(&ci);
    printf("{\"threads\": %d, \"iters\": %d, \"checks\": %ld, \"bad\": %ld, \"errors\": %ld, "
           "\"pattern_entries\": %llu, \"pattern_limit\": %llu, \"uploads\": %llu, \"evictions\": %llu}\n",
           nt, iters, checks, bad, errors, (unsigned long long)ci.pattern_entries,
           (unsigned long long)ci.pattern_entry_limit, (unsigned long long)ci.pattern_uploads,
           (unsigned long long)ci.pattern_evictions);
    return bad || errors ? 1 : 0;
}
