/*
 * tests/glue/drain_recovery_bench.c -- the parity's drain loop while a recovery is in flight
 * (process_rep_command, memcached.c:7739-7767: recovery_try_update_unit, then the parity
 * multiply if it says so), at server level, over the server's own types (rep_queue.h,
 * recovery.h, compiled where they lie).  One JSON line.
 *
 *   drain_recovery_bench [N [SIZE [RANGES [FRAC [REPS]]]]]
 *
 * RS(3,2), this parity P1 (lid 4), D1 lost.  The unchanged server's ecmem: NU = 16,384 units
 * (64 MiB) of host memory.  In flight: RANGES requests of 4 units each (start_recovery's
 * mask P1 + D0 + D2), one every 32 units, each first-touched by D0's reply.  The window: N
 * queued SIZE-byte diffs of D2 at distinct 16-B aligned slots of the arena (live items do
 * not overlap; ecalloc.c:168-229), shuffled, FRAC of them on slots that reach a unit under
 * recovery (D2 has not replied: recovery.c:116-120 folds them there).
 *
 * Paths, each from the same state (restored untimed before every rep), timed over the window:
 *   glue_host   cocytus_drain_gf with cocytus_fold_hook (integration/cocytus_recovery.c: the
 *               units in host memory, every fold of the window in one cec_region_multiply_batch)
 *               into the registered ecmem;
 *   glue_pool   cocytus_drain_gf with cocytus_rpool_fold_hook (cocytus_recovery_pool.c: the
 *               residuals in a pool, every fold in one cec_recovery_pool_fold_updates) into the
 *               registered ecmem;
 *   dropin      the unchanged loop on the shim: per xid the try-update walk with one
 *               galois_w08_region_multiply per unit piece, then one into a pageable ecmem;
 *   cpu         the same loop on the restated CPU region multiply (oracle, SIMD, 1 thread).
 * Checked: every path's arena and unit bytes equal.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <cocytus_ec.h>

#include "cocytus_drain.h"
#include "cocytus_recovery.h"
#include "cocytus_recovery_pool.h"
#include "gf8_ref.h" /* oracle: the restated CPU region multiply (baseline only) */
#include "rep_queue.h"

#define K 3
#define M 2
#define SELF 4
#define NU 16384
#define U ((size_t)UNITSIZE)
#define PEER_REPLIED 0
#define PEER_SET 2

typedef void (*mul_fn)(char *region, int multby, int nbytes, char *r2);
static void mul_dropin(char *region, int c, int n, char *r2) { galois_w08_region_multiply(region, c, n, r2, 1); }
static void mul_cpu(char *region, int c, int n, char *r2) {
    ref_region_multiply_simd((const uint8_t *)region, c, n, (uint8_t *)r2);
}

static int *matrix;
#define MAT(x, y) matrix[(x) * K + (y)]

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    rs ^= rs << 13, rs ^= rs >> 7, rs ^= rs << 17;
    return rs;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint32_t item_nbytes(void *item, void *ctx) {
    (void)ctx;
    return *(uint32_t *)item;
}

/* the fold hooks, timed: how much of a glue path's window is the recovery fold */
static double t_fold;
static int (*inner_hook)(const cec_host_update *, int, int *, void *);
static int timed_hook(const cec_host_update *u, int n, int *need, void *ctx) {
    const double t0 = now_s();
    const int rc = inner_hook(u, n, need, ctx);
    t_fold += now_s() - t0;
    return rc;
}

static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

/* recovery_try_update_unit + the apply, per xid (memcached.c:7758-7767, recovery.c:99-131) */
static void ref_drain(struct recovery *r, char *ecm, const struct rep_queue *q, int n, int size, mul_fn mul) {
    const int c = MAT(SELF, PEER_SET);
    for (int e = 0; e < n; ++e) {
        const struct rep_queue_item *it = &q->items[e];
        uint64_t addr = it->addr;
        uint32_t left = (uint32_t)size;
        const char *d = it->vbuf;
        while (left) {
            const uint64_t off = addr % U, base = addr - off;
            uint32_t len = (uint32_t)(U - off);
            if (left < len) len = left;
            struct recovery_unit *un = &r->units[base / U];
            if ((un->flags & (1u << 30)) && !(un->flags & (1u << PEER_SET)))
                mul((char *)d, c, (int)len, un->data + off);
            addr += len;
            d += len;
            left -= len;
        }
        mul(it->vbuf, c, size, ecm + it->addr); /* (sub_flags NULL: every piece counts) */
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const int size = argc > 2 ? atoi(argv[2]) : 4098;
    const int ranges = argc > 3 ? atoi(argv[3]) : 256;
    const double frac = argc > 4 ? atof(argv[4]) : 0.25;
    const int reps = argc > 5 ? atoi(argv[5]) : 5;
    if (n < 1 || size < 1 || size > (int)(8 * U) || ranges < 1 || ranges * 4 * 8 > NU || reps < 1 || reps > 32)
        return 1;
    if (cec_device_check() != CEC_OK) return fprintf(stderr, "%s\n", cec_last_error()), 2;
    matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    const size_t arena = (size_t)NU * U;
    /* the pristine parity arena, the replying peer's data, the window's diffs */
    char *pristine = malloc(arena), *d0 = malloc(arena);
    for (size_t i = 0; i < arena; i += 8) {
        const uint64_t a = rnd(), b = rnd();
        memcpy(pristine + i, &a, 8);
        memcpy(d0 + i, &b, 8);
    }
    struct rep_queue q;
    q.cap = (uint32_t)n;
    q.items = calloc((size_t)n, sizeof *q.items);
    q.tail = 0;
    q.head = (uint32_t)n;
    uint32_t nbytes = (uint32_t)size;
    /* the slots, split by whether they reach a unit under recovery, each list shuffled */
    const uint64_t stride = ((uint64_t)size + 15) / 16 * 16, n_slots = arena / stride;
    uint64_t *hit = malloc(sizeof(uint64_t) * n_slots), *miss = malloc(sizeof(uint64_t) * n_slots);
    uint64_t nh = 0, nm = 0;
    for (uint64_t sl = 0; sl < n_slots; ++sl) {
        int reaches = 0;
        for (uint64_t u = sl * stride / U; u <= (sl * stride + (uint64_t)size - 1) / U; ++u)
            reaches |= u % 32 < 4 && u / 32 < (uint64_t)ranges;
        if (reaches)
            hit[nh++] = sl;
        else
            miss[nm++] = sl;
    }
    for (uint64_t x = nh; x > 1; --x) {
        const uint64_t y = rnd() % x, tmp = hit[x - 1];
        hit[x - 1] = hit[y];
        hit[y] = tmp;
    }
    for (uint64_t x = nm; x > 1; --x) {
        const uint64_t y = rnd() % x, tmp = miss[x - 1];
        miss[x - 1] = miss[y];
        miss[y] = tmp;
    }
    uint64_t aimed = (uint64_t)(frac * n + 0.5);
    if (aimed > nh) aimed = nh;
    if ((uint64_t)n - aimed > nm) return fprintf(stderr, "%d diffs do not fit the arena's slots\n", n), 1;
    for (int e = 0; e < n; ++e) {
        struct rep_queue_item *it = &q.items[e];
        it->xid = (uint64_t)e + 1;
        it->lid = PEER_SET;
        it->vbuf = malloc((size_t)size);
        for (int b = 0; b < size; ++b) it->vbuf[b] = (char)rnd();
        it->vnbytes = size;
        it->item = &nbytes;
        it->addr = ((uint64_t)e < aimed ? hit[e] : miss[e - aimed]) * stride;
    }
    for (int e = n - 1; e > 0; --e) { /* the aimed ones anywhere in the window */
        const int y = (int)(rnd() % (uint64_t)(e + 1));
        const uint64_t tmp = q.items[e].addr;
        q.items[e].addr = q.items[y].addr;
        q.items[y].addr = tmp;
    }
    free(hit);
    free(miss);
    /* the arenas: two registered (the glue paths), two pageable (the loops) */
    char *ar[4];
    uint8_t *alias[2];
    for (int p = 0; p < 4; ++p)
        if (posix_memalign((void **)&ar[p], 4096, arena)) return 2;
    for (int p = 0; p < 2; ++p)
        if (cec_host_register(ar[p], arena, &alias[p])) return fprintf(stderr, "%s\n", cec_last_error()), 2;
    /* the recovery state: one struct recovery per path (queue items for the pool) */
    struct recovery rec[4];
    struct recovery_queue_item *items = calloc((size_t)ranges, sizeof *items);
    memset(rec, 0, sizeof rec);
    for (int p = 0; p < 4; ++p) rec[p].units = calloc(NU, sizeof(struct recovery_unit));
    rec[1].queue.items = items;
    rec[1].queue.cap = ranges;
    const uint32_t mask = (1u << SELF) | (1u << 0) | (1u << 2);
    for (int q2 = 0; q2 < ranges; ++q2) {
        items[q2].unit_begin = q2 * 32;
        items[q2].unit_end = q2 * 32 + 3;
        items[q2].mask = mask;
    }
    cocytus_rglue *g;
    cocytus_rpool *pg;
    cec_drainer *dr;
    if (cocytus_rglue_create(&g, K, M, matrix, SELF, NULL) ||
        cocytus_rpool_create(&pg, K, M, matrix, SELF, alias[1], ranges, ranges * 4, NULL) ||
        cec_drainer_create(&dr, K, M, matrix, SELF, 64 << 20))
        return fprintf(stderr, "setup: %s\n", cec_last_error()), 2;
    struct ecmem ecm0;
    memset(&ecm0, 0, sizeof ecm0);
    ecm0.mem = ar[0];
    ecm0.size = arena;
    char *touch[K + M];
    for (int l = 0; l < K + M; ++l) touch[l] = calloc(NU, 1);
    cocytus_fold_ctx fc;
    memset(&fc, 0, sizeof fc);
    fc.g = g;
    fc.r = &rec[0];
    for (int l = 0; l < K + M; ++l) fc.touch_flags[l] = touch[l];
    cocytus_rpool_fold_ctx pc;
    memset(&pc, 0, sizeof pc);
    pc.g = pg;
    pc.r = &rec[1];
    for (int l = 0; l < K + M; ++l) pc.touch_flags[l] = touch[l];
    cec_host_update *scratch = calloc((size_t)n, sizeof *scratch);
    double t[4][32], fold_ms[2] = {0, 0};
    for (int path = 0; path < 4; ++path) {
        for (int rep = 0; rep <= reps; ++rep) { /* rep 0: warm-up */
            /* restore: the arena, then every request first-touched by D0's reply */
            memcpy(ar[path], pristine, arena);
            struct recovery *r = &rec[path];
            for (int i = 0; i < NU; ++i) {
                free(r->units[i].data);
                r->units[i].data = NULL;
                r->units[i].flags = 0;
            }
            for (int q2 = 0; q2 < ranges; ++q2) {
                const struct recovery_queue_item *it = &items[q2];
                const char *reply = d0 + (size_t)it->unit_begin * U;
                int rc = 0;
                if (path == 0) {
                    rc = cocytus_recover_units_gf(g, r, &ecm0, PEER_REPLIED, it->unit_begin, it->unit_end, reply);
                } else if (path == 1) {
                    rc = cocytus_rpool_end(pg, r, it);
                    for (int i = it->unit_begin; i <= it->unit_end; ++i) r->units[i].flags = 0;
                    rc = rc ? rc : cocytus_rpool_begin(pg, r, it);
                    rc = rc ? rc : cocytus_rpool_recover_units(pg, r, it, PEER_REPLIED, reply);
                } else {
                    for (int i = it->unit_begin; i <= it->unit_end; ++i) { /* recovery.c:76-93 */
                        struct recovery_unit *un = &r->units[i];
                        un->data = malloc(U);
                        memcpy(un->data, ar[path] + (size_t)i * U, U);
                        un->flags = (1u << 30) | (1u << SELF) | (1u << PEER_REPLIED);
                        (path == 2 ? mul_dropin : mul_cpu)((char *)reply + (size_t)(i - it->unit_begin) * U,
                                                          MAT(SELF, PEER_REPLIED), (int)U, un->data);
                    }
                }
                if (rc) return fprintf(stderr, "restore %d: %d %s\n", path, rc, cec_last_error()), 2;
            }
            if (path == 1 && cocytus_rpool_flush(pg) < 0) return fprintf(stderr, "%s\n", cec_last_error()), 2;
            const double t0 = now_s();
            if (path <= 1) {
                inner_hook = path == 0 ? cocytus_fold_hook : cocytus_rpool_fold_hook;
                cocytus_drain_hooks hooks = {.item_nbytes = item_nbytes, .try_update_batch = timed_hook,
                                             .ctx = path == 0 ? (void *)&fc : (void *)&pc};
                t_fold = 0;
                const int rc = cocytus_drain_gf(&q, PEER_SET, 0, (uint64_t)n, &hooks, dr, alias[path], NULL, scratch, n);
                if (rc != n) return fprintf(stderr, "drain %d: %d %s\n", path, rc, cec_last_error()), 3;
                if (rep) fold_ms[path] += 1e3 * t_fold / reps;
            } else {
                ref_drain(r, ar[path], &q, n, size, path == 2 ? mul_dropin : mul_cpu);
            }
            if (rep) t[path][rep - 1] = now_s() - t0;
            if (path == 2 && rep == 1) { /* the drop-in loop is slow: one timed pass */
                for (int x = 1; x < reps; ++x) t[path][x] = t[path][0];
                break;
            }
        }
        qsort(t[path], (size_t)reps, sizeof(double), cmp_d);
    }
    /* the same bytes everywhere: arenas, and every unit under recovery */
    int ok = 1;
    for (int p = 1; p < 4; ++p) ok &= !memcmp(ar[0], ar[p], arena);
    char *res = malloc(4 * U);
    for (int q2 = 0; q2 < ranges && ok; ++q2) {
        const struct recovery_queue_item *it = &items[q2];
        if (cocytus_rpool_residual(pg, &rec[1], it, res)) return fprintf(stderr, "%s\n", cec_last_error()), 2;
        for (int i = it->unit_begin; i <= it->unit_end; ++i) {
            const char *want = rec[3].units[i].data, *pool_u = res + (size_t)(i - it->unit_begin) * U;
            ok &= !memcmp(rec[0].units[i].data, want, U) && !memcmp(rec[2].units[i].data, want, U) &&
                  !memcmp(pool_u, want, U);
        }
    }
    const double gib = (double)n * size / (double)(1u << 30);
    const double med[4] = {t[0][reps / 2], t[1][reps / 2], t[2][reps / 2], t[3][reps / 2]};
    printf("{\"shape\": \"drain during recovery\", \"diffs\": %d, \"diff_bytes\": %d, \"ranges_in_flight\": %d, "
           "\"units_per_range\": 4, \"aimed_at_recovering_units\": %d, \"arena\": \"host ecmem (64 MiB), registered\", "
           "\"glue_host_ms\": %.3f, \"glue_host_GiBps\": %.2f, \"glue_pool_ms\": %.3f, \"glue_pool_GiBps\": %.2f, "
           "\"dropin_loop_ms\": %.1f, \"dropin_loop_GiBps\": %.3f, \"cpu_restated_1thread_ms\": %.3f, "
           "\"cpu_restated_1thread_GiBps\": %.2f, \"glue_pool_vs_cpu_1thread\": %.2f, \"glue_host_vs_cpu_1thread\": %.2f, "
           "\"glue_pool_vs_dropin\": %.1f, \"fold_hook_ms_mean\": {\"glue_host\": %.3f, \"glue_pool\": %.3f}, "
           "\"reps\": %d, \"verified\": %s}\n",
           n, size, ranges, (int)aimed, 1e3 * med[0], gib / med[0], 1e3 * med[1], gib / med[1], 1e3 * med[2], gib / med[2],
           1e3 * med[3], gib / med[3], med[3] / med[1], med[3] / med[0], med[2] / med[1], fold_ms[0], fold_ms[1], reps,
           ok ? "true" : "false");
    free(res);
    cocytus_rglue_destroy(g);
    cocytus_rpool_destroy(pg);
    cec_drainer_destroy(dr);
    for (int p = 0; p < 2; ++p) cec_host_unregister(ar[p]);
    for (int p = 0; p < 4; ++p) {
        for (int i = 0; i < NU; ++i) free(rec[p].units[i].data);
        free(rec[p].units);
        free(ar[p]);
    }
    for (int e = 0; e < n; ++e) free(q.items[e].vbuf);
    for (int l = 0; l < K + M; ++l) free(touch[l]);
    free(q.items);
    free(items);
    free(scratch);
    free(pristine);
    free(d0);
    free(matrix);
    return ok ? 0 : 4;
}
