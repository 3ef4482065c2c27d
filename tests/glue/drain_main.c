/*
 * tests/glue/drain_main.c -- integration/cocytus_drain.c driven over the server's own
 * queue type: compiled against the reference's rep_queue.h (-I/root/reference; the
 * header is used where it lies, not copied), the way the glue is built in the server tree.
 *
 *   drain_main collect IN OUT   host only: cocytus_drain_collect; OUT = one line per
 *                               collected update "entry addr len lid", or "rc N"
 *   drain_main apply IN OUT     GPU: cocytus_drain_gf into a device parity arena that
 *                               starts from IN's parity bytes; OUT = the arena afterwards
 *   drain_main bench N SIZE [MB [PLACE]]
 *                               GPU: N queued SIZE-byte diffs of one peer drained (a) by
 *                               cocytus_drain_gf into the parity arena, (b) by the unchanged
 *                               loop through the drop-in (one galois_w08_region_multiply
 *                               per xid into a pageable host ecmem, memcached.c:7764), (c) by
 *                               the same loop on the restated CPU region multiply (oracle,
 *                               SIMD, one thread: the reference's GF-Complete path, restated);
 *                               one JSON line.  MB: the drainer's staging (default 64 MiB).
 *                               PLACE: where (a)'s arena lives -- "device" (HBM, default) or
 *                               "host" (the unchanged server's ecmem: host memory registered
 *                               with cec_host_register, the kernels reach it over PCIe)
 *
 * IN (little-endian): int32 lid, self_lid, k, m, ring_cap, tail, n_entries, arena_bytes,
 * cap; uint64 done_xid, stable_xid; n_entries x {uint64 xid, uint64 addr, int32 len,
 * int32 vnbytes, int32 veto}; the entries' diff bytes back to back (len each); then
 * arena_bytes of initial parity.  Entry e sits at ring index tail + e.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <cocytus_ec.h>
#include <galois.h>
#include <reed_sol.h>

#include "cocytus_drain.h"
#include "gf8_ref.h" /* oracle: the restated CPU region multiply (test infrastructure, baseline (c)) */
#include "rep_queue.h"

struct test_item { /* what item_nbytes reads: the test's own value record */
    uint32_t nbytes;
    int veto;
};

static uint32_t item_nbytes(void *item, void *ctx) {
    (void)ctx;
    return ((struct test_item *)item)->nbytes;
}

static int vetoes;     /* try_update calls that kept a diff out of the arena */
static int hook_calls; /* try_update calls */

static int try_update(int lid, uint64_t addr, char *buf, uint32_t nbytes, void *ctx) {
    /* the test's recovery fold: the entry's veto flag, found by its buffer */
    struct test_item *items = ctx;
    (void)lid; (void)addr; (void)nbytes;
    int veto = items[((int32_t *)buf)[-1]].veto; /* entry index stored before the bytes */
    vetoes += veto;
    hook_calls++;
    return !veto;
}

static void rd(FILE *f, void *p, size_t n) {
    if (n && fread(p, 1, n, f) != n) {
        fprintf(stderr, "short input\n");
        exit(3);
    }
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint32_t plain_nbytes(void *item, void *ctx) {
    (void)ctx;
    return *(uint32_t *)item;
}

/* Server-level drain rate: the glue against the unchanged per-xid loop on the shim. */
static int bench(int n, int size, int staging_mb, int host_arena) {
    const int K = 3, M = 2, lid = 1, self = K + 1;
    const size_t arena = (size_t)n * (size_t)size;
    struct rep_queue q;
    q.cap = (uint32_t)n;
    q.items = calloc((size_t)n, sizeof(struct rep_queue_item));
    q.tail = 0;
    q.head = (uint32_t)n;
    uint32_t nbytes = (uint32_t)size;
    uint64_t seed = 0x9E3779B97F4A7C15ull;
    for (int e = 0; e < n; ++e) { /* addresses shuffled over the arena, as ecalloc reuses */
        struct rep_queue_item *it = &q.items[e];
        it->xid = (uint64_t)e + 1;
        it->lid = lid;
        it->vbuf = malloc((size_t)size);
        it->vnbytes = size;
        it->item = &nbytes;
        for (int b = 0; b < size; b += 8) {
            seed ^= seed << 13, seed ^= seed >> 7, seed ^= seed << 17;
            memcpy(it->vbuf + b, &seed, size - b >= 8 ? 8 : (size_t)(size - b));
        }
    }
    for (int e = n - 1; e > 0; --e) { /* Fisher-Yates over the slots */
        seed ^= seed << 13, seed ^= seed >> 7, seed ^= seed << 17;
        const int r = (int)(seed % (uint64_t)(e + 1));
        q.items[e].addr = (uint64_t)r; /* temp: permutation built below */
    }
    int *perm = malloc(sizeof(int) * (size_t)n);
    for (int e = 0; e < n; ++e) perm[e] = e;
    for (int e = n - 1; e > 0; --e) {
        const int r = (int)q.items[e].addr, t = perm[e];
        perm[e] = perm[r];
        perm[r] = t;
    }
    for (int e = 0; e < n; ++e) q.items[e].addr = (uint64_t)perm[e] * (uint64_t)size;
    if (cec_device_check() != CEC_OK) return 2;
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    uint8_t *parity;
    void *slab = NULL;
    uint8_t *host = NULL;
    cec_drainer *dr;
    uint8_t *ecmem = calloc(arena, 1); /* the host ecmem of the unchanged loop; zeros */
    uint8_t *cpu_ecmem = calloc(arena, 1);
    if (host_arena) { /* the server's own host ecmem, registered once */
        if (posix_memalign((void **)&host, 4096, arena) || cec_host_register(memset(host, 0, arena), arena, &parity))
            return 2;
    } else if (cec_arenas_alloc(1, arena, &parity, &slab) || cec_copy(parity, ecmem, arena, NULL) ||
               cec_stream_synchronize(NULL)) {
        return 2;
    }
    if (cec_drainer_create(&dr, K, M, matrix, self, (size_t)staging_mb << 20)) return 2;
    cec_host_update *scratch = calloc((size_t)n, sizeof *scratch);
    cocytus_drain_hooks hooks = {.item_nbytes = plain_nbytes};
    double best = 1e30, t_sum = 0;
    const int reps = 4; /* + one warm-up: 5 drains, an odd count, so the arena holds each diff once */
    for (int r = 0; r < reps + 1; ++r) {
        const double t0 = now_s();
        const int rc = cocytus_drain_gf(&q, lid, 0, (uint64_t)n, &hooks, dr, parity, NULL, scratch, n);
        const double t = now_s() - t0;
        if (rc != n) return 3;
        if (r) {
            t_sum += t;
            if (t < best) best = t;
        }
    }
    /* the unchanged server: one drop-in call per xid into a host ecmem (memcached.c:7764);
     * a first call (and its undo: XOR twice) sets the drop-in's stream and staging up */
    const int c = matrix[self * K + lid];
    galois_w08_region_multiply(q.items[0].vbuf, c, size, (char *)ecmem, 1);
    galois_w08_region_multiply(q.items[0].vbuf, c, size, (char *)ecmem, 1);
    const double t1 = now_s();
    for (int e = 0; e < n; ++e)
        galois_w08_region_multiply(q.items[e].vbuf, c, size, (char *)ecmem + q.items[e].addr, 1);
    const double t_loop = now_s() - t1;
    /* the same loop on the restated CPU path: GF-Complete's split-table SIMD multiply, one
     * thread, into a pageable ecmem (5 passes, like the glue's: each diff applied once) */
    double t_cpu = 1e30;
    for (int r = 0; r < 5; ++r) {
        const double t2 = now_s();
        for (int e = 0; e < n; ++e)
            ref_region_multiply_simd((const uint8_t *)q.items[e].vbuf, c, size, cpu_ecmem + q.items[e].addr);
        const double t = now_s() - t2;
        if (t < t_cpu) t_cpu = t;
    }
    /* every path applied every diff once: the same bytes, and not all zero */
    uint8_t *dev_copy = malloc(arena);
    if (cec_copy(dev_copy, parity, arena, NULL) || cec_stream_synchronize(NULL)) return 2;
    int nonzero = 0;
    for (size_t i = 0; i < arena && !nonzero; ++i) nonzero = ecmem[i] != 0;
    const int ok = nonzero && memcmp(dev_copy, ecmem, arena) == 0 && memcmp(cpu_ecmem, ecmem, arena) == 0 &&
                   (!host || memcmp(host, ecmem, arena) == 0);
    const double gib = (double)arena / (double)(1u << 30);
    printf("{\"path\": \"server drain loop over the real rep_queue: %d queued %d-byte diffs of one peer\", "
           "\"arena\": \"%s\", \"staging_MiB\": %d, "
           "\"glue_GiBps\": %.2f, \"glue_runs\": %d, \"glue_ms_mean\": %.3f, \"glue_ms_best\": %.3f, "
           "\"dropin_loop_GiBps\": %.3f, \"dropin_loop_ms\": %.1f, \"dropin_us_per_xid\": %.2f, "
           "\"cpu_restated_1thread_GiBps\": %.2f, \"cpu_restated_ms_best\": %.3f, "
           "\"speedup_vs_dropin\": %.1f, \"speedup_vs_cpu_1thread\": %.2f, \"launches\": %d, \"verified\": %s}\n",
           n, size, host ? "host ecmem, registered (cec_host_register), reached over PCIe" : "device (HBM)",
           staging_mb, gib / (t_sum / reps), reps, 1e3 * t_sum / reps, 1e3 * best, gib / t_loop, 1e3 * t_loop,
           1e6 * t_loop / n, gib / t_cpu, 1e3 * t_cpu, t_loop / (t_sum / reps), t_cpu / (t_sum / reps),
           cec_drainer_last_launches(dr), ok ? "true" : "false");
    cec_drainer_destroy(dr);
    if (slab) cec_arenas_free(slab);
    if (host) cec_host_unregister(host);
    return ok ? 0 : 4;
}

int main(int argc, char **argv) {
    if (argc >= 4 && argc <= 6 && !strcmp(argv[1], "bench"))
        return bench(atoi(argv[2]), atoi(argv[3]), argc >= 5 ? atoi(argv[4]) : 64,
                     argc == 6 && !strcmp(argv[5], "host"));
    if (argc != 4) return 1;
    /* apply: into a device arena; apply_host: into a registered host arena (the unchanged
     * server's ecmem); apply4k: a drainer with 4 KiB of staging per half, so a window with a
     * larger diff is refused -- before any fold hook runs (cec_drainer_validate) */
    const int host_mode = !strcmp(argv[1], "apply_host"), small = !strcmp(argv[1], "apply4k");
    const int apply = !strcmp(argv[1], "apply") || host_mode || small;
    FILE *in = fopen(argv[2], "rb");
    if (!in) return 1;
    int32_t h[9];
    uint64_t x[2];
    rd(in, h, sizeof h);
    rd(in, x, sizeof x);
    const int lid = h[0], self = h[1], K = h[2], M = h[3], ring = h[4], tail = h[5], n = h[6];
    const size_t arena = (size_t)(uint32_t)h[7];
    const int cap = h[8];
    struct rep_queue q;
    q.cap = (uint32_t)ring;
    q.items = calloc((size_t)ring, sizeof(struct rep_queue_item));
    q.tail = (uint32_t)tail;
    q.head = (uint32_t)(tail + n);
    struct test_item *items = calloc((size_t)n + 1, sizeof *items);
    char *used = calloc((size_t)ring + 1, 1);
    if (n > ring) {
        fprintf(stderr, "%d entries in a ring of %d\n", n, ring);
        return 5;
    }
    for (int e = 0; e < n; ++e) {
        uint64_t xa[2];
        int32_t li[3];
        rd(in, xa, sizeof xa);
        rd(in, li, sizeof li);
        const uint32_t slot = (uint32_t)(tail + e) % q.cap;
        if (used[slot]++) { /* only a ring whose indices wrap 2^32 can do this: not a rep_queue */
            fprintf(stderr, "entry %d reuses ring slot %u\n", e, slot);
            return 5;
        }
        struct rep_queue_item *it = &q.items[slot];
        memset(it, 0, sizeof *it);
        it->xid = xa[0];
        it->lid = lid;
        it->addr = xa[1];
        it->vnbytes = li[1];
        it->item = &items[e];
        items[e].nbytes = (uint32_t)li[0];
        items[e].veto = li[2];
    }
    for (int e = 0; e < n; ++e) { /* each diff in its own malloc'd vbuf, as conn_nread leaves it */
        struct rep_queue_item *it = &q.items[(uint32_t)(tail + e) % q.cap];
        int32_t *blk = malloc(sizeof(int32_t) + (size_t)it->vnbytes + 1);
        blk[0] = e;
        it->vbuf = (char *)(blk + 1);
        rd(in, it->vbuf, items[e].nbytes);
    }
    cocytus_drain_hooks hooks = {.item_nbytes = item_nbytes, .try_update = try_update, .ctx = items};
    cec_host_update *scratch = calloc((size_t)cap + 1, sizeof *scratch);
    FILE *out = fopen(argv[3], apply ? "wb" : "w");
    if (!out) return 1;
    if (!apply) {
        const int rc = cocytus_drain_collect(&q, lid, x[0], x[1], &hooks, scratch, cap);
        if (rc < 0) {
            fprintf(out, "rc %d\n", rc);
        } else {
            for (int i = 0; i < rc; ++i) {
                const int e = ((const int32_t *)scratch[i].buf)[-1];
                fprintf(out, "%d %llu %u %u\n", e, (unsigned long long)scratch[i].addr, scratch[i].len,
                        scratch[i].src_lid);
            }
        }
        fclose(out);
        return 0;
    }
    uint8_t *host = malloc(arena);
    rd(in, host, arena);
    fclose(in);
    if (cec_device_check() != CEC_OK) {
        fprintf(stderr, "%s\n", cec_last_error());
        return 2;
    }
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    uint8_t *parity;
    void *slab = NULL;
    uint8_t *reg = NULL;
    cec_drainer *dr;
    int setup;
    if (host_mode) {
        setup = posix_memalign((void **)&reg, 4096, arena) || !memcpy(reg, host, arena) ||
                cec_host_register(reg, arena, &parity);
    } else {
        setup = cec_arenas_alloc(1, arena, &parity, &slab) || cec_copy(parity, host, arena, NULL) ||
                cec_stream_synchronize(NULL);
    }
    if (setup || cec_drainer_create(&dr, K, M, matrix, self, small ? 4096 : 1 << 20)) {
        fprintf(stderr, "setup: %s\n", cec_last_error());
        return 2;
    }
    const int applied = cocytus_drain_gf(&q, lid, x[0], x[1], &hooks, dr, parity, NULL, scratch, cap);
    if (small) { /* the refusal: no hook ran, the arena is untouched */
        if (cec_copy(host, parity, arena, NULL) || cec_stream_synchronize(NULL)) return 2;
        fwrite(host, 1, arena, out);
        fclose(out);
        printf("rc %d hooks %d\n", applied, hook_calls);
        return 0;
    }
    if (applied < 0) {
        fprintf(stderr, "cocytus_drain_gf: %d %s\n", applied, cec_last_error());
        return 2;
    }
    if (reg) memcpy(host, reg, arena); /* the host arena itself: complete when the drain returned */
    else if (cec_copy(host, parity, arena, NULL) || cec_stream_synchronize(NULL)) return 2;
    fwrite(host, 1, arena, out);
    fclose(out);
    printf("applied %d vetoed %d launches %d\n", applied, vetoes, cec_drainer_last_launches(dr));
    cec_drainer_destroy(dr);
    if (slab) cec_arenas_free(slab);
    if (reg) cec_host_unregister(reg);
    free(matrix);
    return 0;
}
