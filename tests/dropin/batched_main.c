/*
 * tests/dropin/batched_main.c -- the batched bindings of INTEGRATION.md §3, used from C
 * the way server glue would: only <cocytus_ec.h> / <reed_sol.h> and -lcocytus_ec, no HIP
 * header.  RS(K, M) arenas in HBM:
 *   1. encode the data arenas (cec_encode_region)
 *   2. per source shard, one batched fused diff-update with install (cec_diff_update),
 *      the SETs' new values in a device staging buffer
 *   3. the parity drain of the same diffs into a second copy of parity lid K+1 that
 *      started from the encoded parity (cec_drainer_apply, host diffs, overlapping
 *      across shards)
 *   4. D0 lost, leader P0: single-unit recovery requests through a cec_recovery_pool,
 *      replies from host copies of D1..D(K-1), half received in place, rebuilt by
 *      cec_recovery_pool_flush_solve into an out arena
 * The drain and every window of the pool run on a short-lived stream of their own (a
 * connection's), released from the long-lived object before it is destroyed
 * (cec_*_release_stream, the LIFETIME RULE of cocytus_ec.h).
 * Input  (argv[1]): int32 K, M, units, nsets; nsets x int32 (lid, addr, len); the K data
 *        arenas (units x 4096 B each); the SETs' new values back to back.
 * Output (argv[2]): the M parity arenas, the K data arenas after install, the drained
 *        copy of parity K+1, the rebuilt D0 arena.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cocytus_ec.h>
#include <reed_sol.h>

#define U 4096
#define CE(x)                                                                   \
    do {                                                                        \
        int r_ = (x);                                                           \
        if (r_ < 0) {                                                           \
            fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, r_,   \
                    cec_last_error());                                          \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

static void rd(FILE *f, void *p, size_t n) {
    if (fread(p, 1, n, f) != n) {
        fprintf(stderr, "short input\n");
        exit(3);
    }
}

int main(int argc, char **argv) {
    if (argc != 3) return 1;
    FILE *in = fopen(argv[1], "rb");
    if (!in) return 1;
    int32_t hdr[4];
    rd(in, hdr, sizeof hdr);
    const int K = hdr[0], M = hdr[1], units = hdr[2], nsets = hdr[3];
    const size_t A = (size_t)units * U;
    int32_t *sets = malloc(sizeof(int32_t) * 3 * nsets);
    rd(in, sets, sizeof(int32_t) * 3 * nsets);
    uint8_t *host = malloc(A * K);
    rd(in, host, A * K);
    size_t vtotal = 0;
    for (int i = 0; i < nsets; ++i) vtotal += (size_t)sets[3 * i + 2];
    uint8_t *vals = malloc(vtotal + 1);
    rd(in, vals, vtotal);
    fclose(in);

    CE(cec_device_check());
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    /* arenas: K data, M parity, drained parity copy, rebuilt D0 */
    uint8_t *ar[32];
    void *slab;
    CE(cec_arenas_alloc(K + M + 2, A, ar, &slab));
    uint8_t **data = ar, **parity = ar + K, *drained = ar[K + M], *rebuilt = ar[K + M + 1];
    for (int j = 0; j < K; ++j) CE(cec_copy(data[j], host + (size_t)j * A, A, NULL));
    CE(cec_encode_region(K, M, matrix, (const uint8_t *const *)data, parity, A, NULL));
    CE(cec_copy(drained, parity[1], A, NULL));
    CE(cec_stream_synchronize(NULL));

    /* 2. the SETs' values in device staging, one diff-update launch per source shard */
    uint8_t *dstage[2];
    void *sslab;
    CE(cec_arenas_alloc(1, vtotal + 16, dstage, &sslab));
    CE(cec_copy(dstage[0], vals, vtotal, NULL));
    /* the shipped diffs (new ^ stale bytes at the fresh address), for the drain below */
    uint8_t *diffs = malloc(vtotal + 1);
    cec_host_update *ups = malloc(sizeof(cec_host_update) * nsets);
    size_t so = 0;
    for (int i = 0; i < nsets; ++i) {
        const int lid = sets[3 * i], len = sets[3 * i + 2];
        const uint64_t addr = (uint64_t)sets[3 * i + 1];
        for (int b = 0; b < len; ++b) diffs[so + b] = vals[so + b] ^ host[(size_t)lid * A + addr + b];
        ups[i].buf = diffs + so;
        ups[i].addr = addr;
        ups[i].len = (uint32_t)len;
        ups[i].src_lid = (uint32_t)lid;
        so += (size_t)len;
    }
    cec_extent *ext = malloc(sizeof(cec_extent) * nsets);
    for (int j = 0; j < K; ++j) {
        int n = 0;
        so = 0;
        for (int i = 0; i < nsets; ++i) {
            if (sets[3 * i] == j) {
                ext[n].off = (uint64_t)sets[3 * i + 1];
                ext[n].src_off = so;
                ext[n].len = (uint32_t)sets[3 * i + 2];
                ext[n].pattern = (uint32_t)j;
                ++n;
            }
            so += (size_t)sets[3 * i + 2];
        }
        cec_plan *plan;
        CE(cec_plan_create(&plan, ext, n, NULL));
        CE(cec_diff_update(K, M, matrix, data, dstage[0], parity, 1, plan, NULL));
        CE(cec_plan_destroy(plan));
    }

    /* 3. the parity side: drain every diff into the copy of parity K+1 */
    cec_drainer *dr;
    CE(cec_drainer_create(&dr, K, M, matrix, K + 1, 1 << 20));
    void *conn;
    CE(cec_stream_create(&conn));
    CE(cec_drainer_apply(dr, ups, nsets, drained, conn));
    CE(cec_drainer_release_stream(dr, conn));
    CE(cec_stream_destroy(conn));
    CE(cec_drainer_destroy(dr));

    /* 4. D0 lost, leader P0: one request per unit through a pool, replies from host
     *    copies of the (installed) survivors */
    CE(cec_stream_synchronize(NULL));
    uint8_t *live = malloc(A * K);
    for (int j = 0; j < K; ++j) CE(cec_copy(live + (size_t)j * A, data[j], A, NULL));
    CE(cec_stream_synchronize(NULL));
    int connected[32];
    for (int i = 0; i < K + M; ++i) connected[i] = i != 0;
    const uint32_t mask = cec_recovery_mask(K, M, K, connected);
    cec_recovery_pool *pool;
    const int window = 7;
    CE(cec_recovery_pool_create(&pool, K, M, matrix, K, parity[0], window));
    uint8_t *outs[16] = {rebuilt};
    int ids[16];
    for (int base = 0; base < units; base += window) {
        const int w = units - base < window ? units - base : window;
        for (int i = 0; i < w; ++i) {
            ids[i] = cec_recovery_pool_begin(pool, mask, base + i, base + i);
            CE(ids[i]);
            for (int peer = 1; peer < K; ++peer) {
                const uint8_t *src = live + (size_t)peer * A + (size_t)(base + i) * U;
                if ((base + i + peer) % 2) { /* received in place */
                    size_t n;
                    uint8_t *dst = cec_recovery_pool_staging(pool, ids[i], peer, &n);
                    memcpy(dst, src, n);
                    CE(cec_recovery_pool_add_peer(pool, ids[i], peer, dst));
                } else {
                    CE(cec_recovery_pool_add_peer(pool, ids[i], peer, src));
                }
            }
        }
        CE(cec_stream_create(&conn));
        const int solved = cec_recovery_pool_flush_solve(pool, outs, conn);
        CE(solved);
        CE(cec_recovery_pool_release_stream(pool, conn));
        CE(cec_stream_destroy(conn));
        if (solved != w) {
            fprintf(stderr, "solved %d of %d\n", solved, w);
            return 4;
        }
        for (int i = 0; i < w; ++i) CE(cec_recovery_pool_end(pool, ids[i]));
    }
    CE(cec_recovery_pool_destroy(pool));

    /* outputs */
    uint8_t *buf = malloc(A);
    FILE *out = fopen(argv[2], "wb");
    uint8_t *order[64];
    int no = 0;
    for (int p = 0; p < M; ++p) order[no++] = parity[p];
    for (int j = 0; j < K; ++j) order[no++] = data[j];
    order[no++] = drained;
    order[no++] = rebuilt;
    for (int i = 0; i < no; ++i) {
        CE(cec_copy(buf, order[i], A, NULL));
        CE(cec_stream_synchronize(NULL));
        fwrite(buf, 1, A, out);
    }
    fclose(out);
    CE(cec_arenas_free(sslab));
    CE(cec_arenas_free(slab));
    free(buf);
    free(live);
    free(ext);
    free(ups);
    free(diffs);
    free(vals);
    free(host);
    free(sets);
    free(matrix);
    printf("OK\n");
    return 0;
}
