/*
 * tests/dropin/dropin_main.c -- replays the reference's Jerasure call chain through
 * the drop-in headers, linked with -lJerasure (= libcocytus_ec.so).  Written like
 * the Cocytus call sites it mirrors; not a copy of them:
 *   SET on a data server   memcached.c:2667-2681 (diff) + 7762-7767 (each parity) + 5666 (install)
 *   residual per parity    recovery.c:72-94 (first touch copies the parity unit)
 *   leader solve           memcached.c:7880-7922 (jerasure_invert_matrix + n x n multiplies)
 * Input / output are raw little-endian files (see tests/dropin/__init__.py).
 */
#include <galois.h>
#include <jerasure.h>
#include <reed_sol.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define UNIT 4096
#define ALIGN16(p) ((char *)(((uintptr_t)(p) + 15) & ~(uintptr_t)15))

static void rd(FILE *f, void *p, size_t n) {
    if (fread(p, 1, n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
}

int main(int argc, char **argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s in out\n", argv[0]); return 2; }
    FILE *in = fopen(argv[1], "rb");
    if (!in) return 2;
    int32_t hdr[7];
    rd(in, hdr, sizeof hdr);
    const int K = hdr[0], M = hdr[1], arena = hdr[2], nsets = hdr[3], ub = hdr[4], ue = hdr[5];
    const uint32_t mask = (uint32_t)hdr[6];
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    if (!matrix) return 3;
    char *data[32], *parity[32];
    for (int j = 0; j < K; ++j) data[j] = calloc(arena, 1);
    for (int p = 0; p < M; ++p) parity[p] = calloc(arena, 1);
    int32_t *sets = malloc(sizeof(int32_t) * 3 * (nsets > 0 ? nsets : 1));
    rd(in, sets, sizeof(int32_t) * 3 * nsets);
    for (int s = 0; s < nsets; ++s) {
        const int j = sets[3 * s], addr = sets[3 * s + 1], n = sets[3 * s + 2];
        char *vbuf = malloc(n);
        rd(in, vbuf, n);
        char *old = data[j] + addr;
        char *diff_base = malloc(n + 15 + 128);
        char *diff = ALIGN16(diff_base);
        memcpy(diff, vbuf, n);
        galois_w08_region_multiply(old, 1, n, diff, 1);
        for (int p = 0; p < M; ++p)
            galois_w08_region_multiply(diff, matrix[(K + p) * K + j], n, parity[p] + addr, 1);
        memcpy(old, vbuf, n);
        free(diff_base);
        free(vbuf);
    }
    fclose(in);

    /* online recovery of units [ub, ue] with participant mask */
    const int nunits = ue - ub + 1, nbuf = nunits * UNIT;
    int n = 0;
    for (int j = 0; j < K; ++j) if (!(mask & (1u << j))) ++n;
    char *C[32];
    int *tmpmat = malloc(sizeof(int) * (n * n + 1)), nn = 0, m = 0;
    for (int p = K; p < K + M; ++p) {
        if (!(mask & (1u << p))) continue;
        char **units = calloc(nunits, sizeof(char *));
        for (int s = 0; s < K; ++s) {          /* one recover_units_reply per data peer */
            if (!(mask & (1u << s))) continue;
            for (int u = 0; u < nunits; ++u) {
                if (!units[u]) {
                    units[u] = malloc(UNIT);
                    memcpy(units[u], parity[p - K] + (size_t)(ub + u) * UNIT, UNIT);
                }
                galois_w08_region_multiply(data[s] + (size_t)(ub + u) * UNIT, matrix[p * K + s], UNIT,
                                           units[u], 1);
            }
        }
        char *buf = malloc(nbuf);
        for (int u = 0; u < nunits; ++u) {
            if (!units[u]) { units[u] = malloc(UNIT); memcpy(units[u], parity[p - K] + (size_t)(ub + u) * UNIT, UNIT); }
            memcpy(buf + (size_t)u * UNIT, units[u], UNIT);
            free(units[u]);
        }
        free(units);
        C[m++] = buf;
        for (int j = 0; j < K; ++j)
            if (!(mask & (1u << j))) tmpmat[nn++] = matrix[p * K + j];
    }
    if (m != n || nn != n * n) { fprintf(stderr, "bad mask\n"); return 4; }
    int *inv = malloc(sizeof(int) * (n * n + 1));
    if (n && jerasure_invert_matrix(tmpmat, inv, n, 8) != 0) { fprintf(stderr, "singular\n"); return 5; }
    char *rec[32];
    for (int i = 0; i < n; ++i) {
        rec[i] = calloc(nbuf, 1);
        for (int x = 0; x < n; ++x) galois_w08_region_multiply(C[x], inv[i * n + x], nbuf, rec[i], 1);
    }
    FILE *out = fopen(argv[2], "wb");
    for (int j = 0; j < K; ++j) fwrite(data[j], 1, arena, out);
    for (int p = 0; p < M; ++p) fwrite(parity[p], 1, arena, out);
    for (int i = 0; i < n; ++i) fwrite(rec[i], 1, nbuf, out);
    fclose(out);
    for (int i = 0; i < n; ++i) free(rec[i]);
    for (int i = 0; i < m; ++i) free(C[i]);
    for (int j = 0; j < K; ++j) free(data[j]);
    for (int p = 0; p < M; ++p) free(parity[p]);
    free(inv);
    free(tmpmat);
    free(sets);
    free(matrix); /* the server never frees it (memcached.c:6845); a test does */
    printf("dropin ok: K=%d M=%d sets=%d units=%d lost=%d\n", K, M, nsets, nunits, n);
    return 0;
}
