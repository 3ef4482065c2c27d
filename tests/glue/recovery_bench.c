/*
 * tests/glue/recovery_bench.c -- the recovery glue (integration/cocytus_recovery.c) against
 * the unchanged server's per-unit code, at server level, over the server's own types
 * (compiled against the reference's recovery.h / ecmem.h where they lie).
 *
 *   recovery_bench [REPS]      one JSON line per shape:
 *   recovery_bench set N SIZE [REPS]
 *               the data side (integration/cocytus_set.c): the diffs of N SETs of SIZE bytes
 *               (complete_nread, memcached.c:2664-2681) at shuffled 16-B aligned addresses of a
 *               host ecmem, values in their own malloc'd buffers: one cocytus_set_diffs_gf
 *               against the per-SET drop-in call and the restated CPU call (1 thread).
 *
 * Every rep recovers other units (32 MiB further into a host arena of (REPS + 2) x 32 MiB), so
 * the parity bytes of the first touch come cold from memory in every path, as they do when a
 * recovery walks the arena; the replies are hot (just received).
 *
 *   range_1MiB  one recovery request over 256 units (1 MiB), RS(3,2), this parity P1 the
 *               leader of a single loss (D1 lost; mask P1 + D0 + D2, start_recovery's):
 *               two data peers' replies (recovery_recover_units, recovery.c:61-96), then
 *               the leader solve (complete_recovery_bottom_half, memcached.c:7842-7922).
 *   idle_85     the idle recoverer's 85 single-unit requests in flight (idle_event_handler,
 *               memcached.c:5712-5734; TOO_MANY_RECOVERY, const.h:27) at scattered units:
 *               2 replies each, then 85 leader solves.
 *
 * Paths, all from the same inputs, outputs compared byte for byte:
 *   glue        cocytus_recover_units_gf x peers + cocytus_recovery_solve_gf (range), or
 *               every reply and solve deferred and ONE cocytus_recovery_flush (idle);
 *   pool        the pool placement (integration/cocytus_recovery_pool.c): every request
 *               begun, every reply copied into the pool's staging, every solve queued, ONE
 *               cocytus_rpool_flush (one launch); fill_completed_recovered_data then reads
 *               the rebuilt bytes in place in the pool's mapped output, as it reads the other
 *               paths' data[] (that memcpy and recovery_req_remove are untimed in every path);
 *   pool_recv_in_staging  the same with every reply received straight into the pool's
 *               staging (cocytus_rpool_staging as c->ritem): the recv, like every other
 *               path's recv into c->vbuf, is not timed, so no copy is;
 *   dropin      the reference's loops as the unchanged server runs them on the shim: one
 *               synchronous galois_w08_region_multiply per unit (and per solve term);
 *   cpu         the same loops on the restated CPU region multiply (oracle: GF-Complete's
 *               split-table SIMD, one thread) -- the reference's own CPU path, restated.
 * The recovery state and the arena are host memory in every path (the unchanged server's).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <cocytus_ec.h>

#include "cocytus_recovery.h"
#include "cocytus_recovery_pool.h"
#include "cocytus_set.h"
#include "gf8_ref.h" /* oracle: the restated CPU region multiply (baseline only) */

#define K 3
#define M 2
#define SELF 4 /* P1 */
#define U ((size_t)UNITSIZE)

typedef void (*mul_fn)(char *region, int multby, int nbytes, char *r2);

static void mul_dropin(char *region, int c, int n, char *r2) { galois_w08_region_multiply(region, c, n, r2, 1); }
static void mul_cpu(char *region, int c, int n, char *r2) {
    ref_region_multiply_simd((const uint8_t *)region, c, n, (uint8_t *)r2);
}

static int *matrix;
#define MAT(x, y) matrix[(x) * K + (y)]
static int register_ecmem = 1; /* RECOVERY_BENCH_STAGED=1: leave ecmem unregistered (every base staged) */

/* recovery_recover_units (recovery.c:61-96), per unit */
static void ref_recover(struct recovery *r, struct ecmem *ecm, int peer, int ub, int ue, char *data, mul_fn mul) {
    for (int i = ub; i <= ue; ++i, data += U) {
        struct recovery_unit *u = &r->units[i];
        if (!(u->flags & (1u << 30))) {
            u->data = malloc(U);
            memcpy(u->data, ecmem_get(ecm, (uint64_t)i * U), U);
            u->flags |= (1u << 30) | (1u << SELF);
        }
        u->flags |= 1u << peer;
        mul(data, MAT(SELF, peer), (int)U, u->data);
    }
}

/* complete_recovery_bottom_half's arithmetic (memcached.c:7842-7922) for a single loss led
 * by this parity: buf = the units copied out, data = calloc, data ^= inv * buf */
static char *ref_solve(struct recovery *r, int ub, int ue, int inv, mul_fn mul) {
    const size_t nbuf = (size_t)(ue - ub + 1) * U;
    char *buf = malloc(nbuf), *p = buf;
    for (int i = ub; i <= ue; ++i, p += U) memcpy(p, r->units[i].data, U);
    char *out = calloc(1, nbuf);
    mul(buf, inv, (int)nbuf, out);
    free(buf);
    return out;
}

enum { kRepStride = 8192 }; /* units (32 MiB) between the ranges of consecutive reps */

static void reset(struct recovery *r, int nunits) {
    for (int i = 0; i < nunits; ++i) {
        if (!r->units[i].data && !r->units[i].flags) continue;
        free(r->units[i].data);
        r->units[i].data = NULL;
        r->units[i].flags = 0;
    }
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static void fill(char *p, size_t n, uint64_t seed) {
    for (size_t i = 0; i < n; i += 8) {
        seed ^= seed << 13, seed ^= seed >> 7, seed ^= seed << 17;
        memcpy(p + i, &seed, n - i >= 8 ? 8 : n - i);
    }
}

/* One shape: nreq requests of `units` units each at unit starts[q]. */
static int shape(const char *name, int nreq, int units, const int *starts, int reps, int nunits, struct ecmem *ecm,
                 cocytus_rglue *g, const uint8_t *alias) {
    const int peers[2] = {0, 2}, lost = 1;
    const uint32_t mask = (1u << SELF) | (1u << 0) | (1u << 2);
    const int inv = galois_single_divide(1, MAT(SELF, lost), 8);
    const size_t nbuf = (size_t)units * U;
    struct recovery r;
    memset(&r, 0, sizeof r);
    r.units = calloc((size_t)nunits, sizeof *r.units);
    char **reply = malloc(sizeof(char *) * (size_t)(2 * nreq)); /* c->vbuf of each reply */
    for (int x = 0; x < 2 * nreq; ++x) {
        reply[x] = malloc(nbuf);
        fill(reply[x], nbuf, 0x1234567ull + (uint64_t)x);
    }
    char **out[5];
    for (int p = 0; p < 5; ++p) out[p] = calloc((size_t)nreq, sizeof(char *));
    const char **pdata = calloc((size_t)nreq, sizeof *pdata);
    double t[5][64];
    struct recovery_queue_item *it = calloc((size_t)nreq, sizeof *it);
    for (int q = 0; q < nreq; ++q) it[q].mask = mask;
    r.queue.items = it; /* the requests' keys in the pool placement */
    r.queue.cap = nreq;
    cocytus_rpool *pg = NULL; /* needs the arena's device view: a registered ecmem */
    if (alias && cocytus_rpool_create(&pg, K, M, matrix, SELF, alias, nreq, nreq * units, NULL))
        return fprintf(stderr, "rpool: %s\n", cec_last_error()), 2;
    const int npath = pg ? 5 : 3;
    for (int path = 0; path < npath; ++path) {
        for (int rep = 0; rep <= reps; ++rep) { /* rep 0: warm-up */
            reset(&r, nunits);
            for (int q = 0; q < nreq; ++q) free(out[path][q]);
            /* each rep recovers other units of the arena (32 MiB further on), so their parity
             * bytes come cold from host memory, as a recovery scanning the arena reads them */
            for (int q = 0; q < nreq; ++q) {
                it[q].unit_begin = starts[q] + rep * kRepStride;
                it[q].unit_end = it[q].unit_begin + units - 1;
            }
            if (path == 4) { /* the recv: each reply read into the pool's staging (c->ritem), untimed
                                as every other path's recv into c->vbuf */
                for (int q = 0; q < nreq; ++q)
                    if (cocytus_rpool_begin(pg, &r, &it[q])) return fprintf(stderr, "begin: %s\n", cec_last_error()), 2;
                for (int q = 0; q < nreq; ++q)
                    for (int p = 0; p < 2; ++p) memcpy(cocytus_rpool_staging(pg, &r, &it[q], peers[p]), reply[2 * q + p], nbuf);
            }
            const double t0 = now_s();
            double t_end = 0;
            if (path == 0) {
                for (int q = 0; q < nreq; ++q)
                    for (int p = 0; p < 2; ++p) {
                        const int rc = nreq == 1 ? cocytus_recover_units_gf(g, &r, ecm, peers[p], it[q].unit_begin,
                                                                            it[q].unit_end, reply[2 * q + p])
                                                 : cocytus_recover_units_defer(g, &r, ecm, peers[p], it[q].unit_begin,
                                                                               it[q].unit_end, reply[2 * q + p], 0);
                        if (rc) return fprintf(stderr, "recover: %d %s\n", rc, cec_last_error()), 2;
                    }
                for (int q = 0; q < nreq; ++q) {
                    char *data[M];
                    int n = 0;
                    const int rc = nreq == 1 ? cocytus_recovery_solve_gf(g, &r, &it[q], data, &n)
                                             : cocytus_recovery_solve_defer(g, &r, &it[q], data, &n);
                    if (rc || n != 1) return fprintf(stderr, "solve: %d %s\n", rc, cec_last_error()), 2;
                    out[0][q] = data[0];
                }
                if (nreq > 1 && cocytus_recovery_flush(g) != 3 * nreq)
                    return fprintf(stderr, "flush: %s\n", cec_last_error()), 2;
            } else if (path >= 3) {
                if (path == 3)
                    for (int q = 0; q < nreq; ++q)
                        if (cocytus_rpool_begin(pg, &r, &it[q]))
                            return fprintf(stderr, "begin: %s\n", cec_last_error()), 2;
                for (int q = 0; q < nreq; ++q)
                    for (int p = 0; p < 2; ++p) {
                        const char *src = path == 3 ? reply[2 * q + p] : cocytus_rpool_staging(pg, &r, &it[q], peers[p]);
                        if (cocytus_rpool_recover_units(pg, &r, &it[q], peers[p], src))
                            return fprintf(stderr, "reply: %s\n", cec_last_error()), 2;
                    }
                for (int q = 0; q < nreq; ++q) {
                    int n = 0;
                    if (cocytus_rpool_solve(pg, &r, &it[q], &n) || n != 1)
                        return fprintf(stderr, "solve: %s\n", cec_last_error()), 2;
                }
                if (cocytus_rpool_flush(pg) != nreq) return fprintf(stderr, "flush: %s\n", cec_last_error()), 2;
                for (int q = 0; q < nreq; ++q) pdata[q] = cocytus_rpool_data(pg, &r, &it[q], 0);
                t_end = now_s(); /* fill_completed_recovered_data reads data in place from here on, as it
                                    reads the other paths' data[] */
                for (int q = 0; q < nreq; ++q) {
                    out[path][q] = malloc(nbuf);
                    memcpy(out[path][q], pdata[q], nbuf);
                    cocytus_rpool_end(pg, &r, &it[q]); /* recovery_req_remove (untimed in every path) */
                    for (int i = it[q].unit_begin; i <= it[q].unit_end; ++i) r.units[i].flags = 0;
                }
            } else {
                const mul_fn mul = path == 1 ? mul_dropin : mul_cpu;
                for (int q = 0; q < nreq; ++q)
                    for (int p = 0; p < 2; ++p)
                        ref_recover(&r, ecm, peers[p], it[q].unit_begin, it[q].unit_end, reply[2 * q + p], mul);
                for (int q = 0; q < nreq; ++q) out[path][q] = ref_solve(&r, it[q].unit_begin, it[q].unit_end, inv, mul);
            }
            if (rep) t[path][rep - 1] = (path >= 3 ? t_end : now_s()) - t0;
        }
        qsort(t[path], (size_t)reps, sizeof(double), cmp_d);
    }
    int same = 1;
    for (int q = 0; q < nreq; ++q)
        same &= !memcmp(out[0][q], out[1][q], nbuf) && !memcmp(out[0][q], out[2][q], nbuf) &&
                (!pg || (!memcmp(out[0][q], out[3][q], nbuf) && !memcmp(out[0][q], out[4][q], nbuf)));
    /* payload: the replies folded + the bytes rebuilt */
    const double bytes = (double)nreq * (double)nbuf * 3.0, gib = bytes / (double)(1u << 30);
    const double med[5] = {t[0][reps / 2], t[1][reps / 2], t[2][reps / 2], pg ? t[3][reps / 2] : 0.0,
                           pg ? t[4][reps / 2] : 0.0};
    cec_batch_stats st;
    cec_region_multiply_batch_stats(&st);
    printf("{\"shape\": \"%s\", \"requests\": %d, \"units_per_request\": %d, \"code\": \"RS(3,2), leader P1, D1 lost\", "
           "\"payload_MiB\": %.3f, \"glue_us\": %.1f, \"glue_GiBps\": %.3f, \"dropin_loop_us\": %.1f, "
           "\"dropin_loop_GiBps\": %.3f, \"cpu_restated_1thread_us\": %.1f, \"cpu_restated_1thread_GiBps\": %.3f, "
           "\"glue_vs_dropin\": %.1f, \"glue_vs_cpu_1thread\": %.2f, \"pool_us\": %.1f, \"pool_GiBps\": %.3f, "
           "\"pool_vs_cpu_1thread\": %.2f, \"pool_vs_glue\": %.2f, \"pool_recv_in_staging_us\": %.1f, "
           "\"pool_recv_in_staging_GiBps\": %.3f, \"pool_recv_in_staging_vs_cpu_1thread\": %.2f, \"reps\": %d, "
           "\"ecmem_registered\": %d, \"last_batch\": {\"launches\": %d, \"in_place\": %d, \"pack_us\": %.1f, \"gpu_us\": %.1f, \"unpack_us\": %.1f}, "
           "\"verified\": %s}\n",
           name, nreq, units, bytes / (1 << 20), 1e6 * med[0], gib / med[0], 1e6 * med[1], gib / med[1], 1e6 * med[2],
           gib / med[2], med[1] / med[0], med[2] / med[0], 1e6 * med[3], pg ? gib / med[3] : 0.0,
           pg ? med[2] / med[3] : 0.0, pg ? med[0] / med[3] : 0.0, 1e6 * med[4], pg ? gib / med[4] : 0.0,
           pg ? med[2] / med[4] : 0.0, reps, register_ecmem, st.launches, st.in_place_launches,
           st.pack_us, st.gpu_us, st.unpack_us,
           same ? "true" : "false");
    reset(&r, nunits);
    cocytus_rpool_destroy(pg);
    for (int p = 0; p < 5; ++p) {
        for (int q = 0; q < nreq; ++q) free(out[p][q]);
        free(out[p]);
    }
    free(pdata);
    for (int x = 0; x < 2 * nreq; ++x) free(reply[x]);
    free(reply);
    free(it);
    free(r.units);
    return same ? 0 : 4;
}

static int set_bench(int n, int size, int reps) {
    const size_t stride = ((size_t)size + 15) / 16 * 16, arena = (size_t)n * stride;
    struct ecmem ecm;
    memset(&ecm, 0, sizeof ecm);
    ecm.size = arena;
    ecm.mem = malloc(arena);
    fill(ecm.mem, arena, 5);
    uint8_t *alias; /* the data process's ecmem registered once, as INTEGRATION §3 sets it up:
                       the batch reads the old bytes in place */
    if (register_ecmem && cec_host_register(ecm.mem, arena, &alias)) return fprintf(stderr, "%s\n", cec_last_error()), 2;
    cocytus_set_diff *sd = calloc((size_t)n, sizeof *sd);
    int *perm = malloc(sizeof(int) * (size_t)n);
    for (int e = 0; e < n; ++e) perm[e] = e;
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int e = n - 1; e > 0; --e) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        const int r = (int)(s % (uint64_t)(e + 1)), t = perm[e];
        perm[e] = perm[r];
        perm[r] = t;
    }
    char *diffs[3];
    for (int p = 0; p < 3; ++p) diffs[p] = malloc((size_t)n * stride);
    for (int e = 0; e < n; ++e) {
        char *v = malloc((size_t)size);
        fill(v, (size_t)size, 1000 + (uint64_t)e);
        sd[e].value = v;
        sd[e].addr = (uint64_t)perm[e] * stride;
        sd[e].nbytes = (uint32_t)size;
    }
    double t[3][64];
    for (int path = 0; path < 3; ++path) {
        for (int e = 0; e < n; ++e) sd[e].diff = diffs[path] + (size_t)e * stride;
        for (int rep = 0; rep <= reps; ++rep) {
            const double t0 = now_s();
            if (path == 0) {
                if (cocytus_set_diffs_gf(&ecm, sd, n, NULL)) return fprintf(stderr, "%s\n", cec_last_error()), 2;
            } else {
                for (int e = 0; e < n; ++e) { /* memcached.c:2676-2681 */
                    memcpy(sd[e].diff, sd[e].value, (size_t)size);
                    char *old = ecmem_get(&ecm, sd[e].addr);
                    if (path == 1) galois_w08_region_multiply(old, 1, size, sd[e].diff, 1);
                    else ref_region_multiply_simd((const uint8_t *)old, 1, size, (uint8_t *)sd[e].diff);
                }
            }
            if (rep) t[path][rep - 1] = now_s() - t0;
            if (path == 1 && rep == 1) { /* the drop-in loop is slow: one timed pass */
                t[path][1] = t[path][0];
                break;
            }
        }
        qsort(t[path], (size_t)(path == 1 ? 2 : reps), sizeof(double), cmp_d);
    }
    int same = 1;
    for (int e = 0; e < n; ++e)
        same &= !memcmp(diffs[0] + (size_t)e * stride, diffs[1] + (size_t)e * stride, (size_t)size) &&
                !memcmp(diffs[0] + (size_t)e * stride, diffs[2] + (size_t)e * stride, (size_t)size);
    const double gib = (double)n * size / (double)(1u << 30);
    const double med[3] = {t[0][reps / 2], t[1][0], t[2][reps / 2]};
    cec_batch_stats st;
    cec_region_multiply_batch_stats(&st);
    printf("{\"shape\": \"set_diffs\", \"sets\": %d, \"value_bytes\": %d, \"glue_ms\": %.3f, \"glue_GiBps\": %.2f, "
           "\"dropin_loop_ms\": %.1f, \"dropin_loop_GiBps\": %.3f, \"dropin_us_per_set\": %.2f, "
           "\"cpu_restated_1thread_ms\": %.3f, \"cpu_restated_1thread_GiBps\": %.2f, \"glue_vs_dropin\": %.1f, "
           "\"glue_vs_cpu_1thread\": %.2f, \"ecmem_registered\": %d, \"last_batch\": {\"launches\": %d, \"in_place\": %d, \"rounds\": %d, \"plan_us\": %.0f, "
           "\"pack_us\": %.0f, \"gpu_wait_us\": %.0f, \"unpack_us\": %.0f}, \"verified\": %s}\n",
           n, size, 1e3 * med[0], gib / med[0], 1e3 * med[1], gib / med[1], 1e6 * med[1] / n, 1e3 * med[2],
           gib / med[2], med[1] / med[0], med[2] / med[0], register_ecmem, st.launches, st.in_place_launches, st.rounds,
           st.plan_us, st.pack_us, st.gpu_us,
           st.unpack_us, same ? "true" : "false");
    for (int e = 0; e < n; ++e) free((void *)sd[e].value);
    for (int p = 0; p < 3; ++p) free(diffs[p]);
    free(sd);
    free(perm);
    if (register_ecmem) cec_host_unregister(ecm.mem);
    free(ecm.mem);
    return same ? 0 : 4;
}

int main(int argc, char **argv) {
    register_ecmem = !(getenv("RECOVERY_BENCH_STAGED") && atoi(getenv("RECOVERY_BENCH_STAGED")));
    if (argc >= 4 && !strcmp(argv[1], "set")) {
        if (cec_device_check() != CEC_OK) return fprintf(stderr, "%s\n", cec_last_error()), 2;
        const int reps = argc > 4 ? atoi(argv[4]) : 7;
        if (reps < 1 || reps > 64) return 1;
        return set_bench(atoi(argv[2]), atoi(argv[3]), reps);
    }
    const int reps = argc > 1 ? atoi(argv[1]) : 15;
    if (reps < 1 || reps > 64) return 1;
    if (cec_device_check() != CEC_OK) return fprintf(stderr, "%s\n", cec_last_error()), 2;
    matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    /* a (reps + 2) x 32 MiB parity arena, host memory (the server's ecmem), walked in 32 MiB steps */
    const int nunits = 8192 * (reps + 1) + 8192;
    struct ecmem ecm;
    memset(&ecm, 0, sizeof ecm);
    ecm.size = (uint64_t)nunits * U;
    ecm.mem = malloc(ecm.size);
    fill(ecm.mem, ecm.size, 99);
    uint8_t *alias; /* the parity's ecmem registered once (the drain needs it so):
                       the first-touch parity units are then read in place */
    if (register_ecmem && cec_host_register(ecm.mem, ecm.size, &alias)) return fprintf(stderr, "%s\n", cec_last_error()), 2;
    cocytus_rglue *g;
    if (cocytus_rglue_create(&g, K, M, matrix, SELF, NULL)) return 2;
    int start = 100;
    const uint8_t *dev_view = register_ecmem ? alias : NULL;
    int rc = shape("range_1MiB", 1, 256, &start, reps, nunits, &ecm, g, dev_view);
    int starts[85];
    uint64_t s = 77;
    for (int q = 0; q < 85; ++q) { /* distinct scattered units */
        int ok;
        do {
            s ^= s << 13, s ^= s >> 7, s ^= s << 17;
            starts[q] = 512 + (int)(s % (uint64_t)(kRepStride - 512)); /* scattered in the rep's 32 MiB */
            ok = 1;
            for (int x = 0; x < q; ++x) ok &= starts[x] != starts[q];
        } while (!ok);
    }
    rc |= shape("idle_85", 85, 1, starts, reps, nunits, &ecm, g, dev_view);
    cocytus_rglue_destroy(g);
    if (register_ecmem) cec_host_unregister(ecm.mem);
    free(ecm.mem);
    free(matrix);
    return rc;
}
