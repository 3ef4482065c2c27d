/*
 * tools/bench_native.c -- bench.py's metric step driven through the C-ABI alone: a C99
 * program with no HIP header, no Python and no torch, linked -lcocytus_ec.  It shows
 * the library is the product and torch only plumbing (not product; a cross-check).
 *
 * RS(3,2), 65,536 stripes of 4 KiB in arenas from cec_arenas_alloc (odd-4 KiB stride),
 * data filled from the host with splitmix64 bytes (cec_copy), one encode + one decode
 * per step, the lost data shard and the leader rotating over all (lost, leader) pairs
 * as in bench.py (masks from cec_recovery_mask = start_recovery, memcached.c:8136-8151),
 * one event between consecutive launches, W warm-up steps then S timed steps.  Every
 * rebuilt shard is compared with its original.  Prints one JSON line.
 *   make -C tools   (needs cocytus_amd/libcocytus_ec.so)
 */
#include <cocytus_ec.h>
#include <reed_sol.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define CE(x)                                                               \
    do {                                                                    \
        int r_ = (x);                                                       \
        if (r_ < 0) {                                                       \
            fprintf(stderr, "%s: %d %s\n", #x, r_, cec_last_error());       \
            return 1;                                                       \
        }                                                                   \
    } while (0)

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char **argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 20, W = argc > 2 ? atoi(argv[2]) : 3;
    enum { K = 3, M = 2, NMASK = K * M };
    const size_t n = 4096, B = 65536, L = n * B;
    CE(cec_device_check());
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    if (!matrix) return 1;
    uint8_t *ar[K + M + K];
    void *slab = NULL;
    CE(cec_arenas_alloc(K + M + K, L, ar, &slab));
    uint8_t *data[K] = {ar[0], ar[1], ar[2]}, *parity[M] = {ar[3], ar[4]};
    uint8_t *out[K] = {ar[5], ar[6], ar[7]};
    const uint8_t *survivors[K + M] = {ar[0], ar[1], ar[2], ar[3], ar[4]};

    uint8_t *h = malloc(L);
    uint64_t x = 0xC0C70002ull;
    for (int j = 0; j < K; ++j) {
        for (size_t i = 0; i < L; i += 8) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            memcpy(h + i, &z, 8);
        }
        CE(cec_copy(data[j], h, L, NULL));
        CE(cec_stream_synchronize(NULL));
    }

    uint32_t masks[NMASK];
    int lost_of[NMASK];
    for (int p = 0; p < M; ++p)
        for (int j = 0; j < K; ++j) {
            int conn[K + M];
            for (int i = 0; i < K + M; ++i) conn[i] = i != j;
            masks[p * K + j] = cec_recovery_mask(K, M, K + p, conn);
            lost_of[p * K + j] = j;
        }
    cec_extent *ext = malloc(sizeof(cec_extent) * B);
    for (size_t s = 0; s < B; ++s) {
        ext[s].off = s * n;
        ext[s].src_off = 0;
        ext[s].len = (uint32_t)n;
        ext[s].pattern = 0;
    }
    cec_plan *ep, *dp;
    CE(cec_plan_create(&ep, ext, (int)B, NULL));
    for (size_t s = 0; s < B; ++s) ext[s].pattern = (uint32_t)(s % NMASK);
    CE(cec_plan_create(&dp, ext, (int)B, NULL));

    for (int w = 0; w < W; ++w) {
        CE(cec_encode(K, M, matrix, (const uint8_t *const *)data, parity, ep, NULL));
        CE(cec_decode(K, M, matrix, masks, NMASK, survivors, out, dp, NULL));
    }
    CE(cec_stream_synchronize(NULL));

    void **ev = malloc(sizeof(void *) * (size_t)(2 * S + 1));
    for (int i = 0; i < 2 * S + 1; ++i) CE(cec_event_create(&ev[i]));
    const double t0 = now();
    CE(cec_event_record(ev[0], NULL));
    for (int s = 0; s < S; ++s) {
        CE(cec_encode(K, M, matrix, (const uint8_t *const *)data, parity, ep, NULL));
        CE(cec_event_record(ev[2 * s + 1], NULL));
        CE(cec_decode(K, M, matrix, masks, NMASK, survivors, out, dp, NULL));
        CE(cec_event_record(ev[2 * s + 2], NULL));
    }
    CE(cec_stream_synchronize(NULL));
    const double el = now() - t0;
    double enc = 0, dec = 0;
    for (int s = 0; s < S; ++s) {
        float a, b;
        CE(cec_event_elapsed_ms(ev[2 * s], ev[2 * s + 1], &a));
        CE(cec_event_elapsed_ms(ev[2 * s + 1], ev[2 * s + 2], &b));
        enc += a;
        dec += b;
    }
    enc /= S;
    dec /= S;

    /* verify: every stripe's rebuilt shard equals the original */
    uint8_t *got = malloc(L), *want = malloc(L);
    size_t bad = 0;
    for (int j = 0; j < K; ++j) {
        CE(cec_copy(got, out[j], L, NULL));
        CE(cec_copy(want, data[j], L, NULL));
        CE(cec_stream_synchronize(NULL));
        for (size_t s = 0; s < B; ++s)
            if (lost_of[s % NMASK] == j && memcmp(got + s * n, want + s * n, n) != 0) ++bad;
    }
    const double payload = (double)(K + 1) * (double)L * S;
    printf("{\"metric\": \"GiB/s device-resident RS(3,2) encode+decode, 4 KiB values\", "
           "\"harness\": \"tools/bench_native.c (C-ABI only, no Python / torch)\", "
           "\"value\": %.2f, \"unit\": \"GiB/s\", \"steps\": %d, \"warmup\": %d, "
           "\"ms_per_step\": %.4f, \"encode_ms\": %.4f, \"encode_frac\": %.4f, "
           "\"decode_ms\": %.4f, \"decode_frac\": %.4f, \"verified\": %s}\n",
           payload / el / (double)(1u << 30), S, W, el * 1e3 / S, enc,
           (double)(K + M) * (double)L / (enc * 1e-3) / 8e12, dec,
           (double)(K + 1) * (double)L / (dec * 1e-3) / 8e12, bad ? "false" : "true");
    for (int i = 0; i < 2 * S + 1; ++i) cec_event_destroy(ev[i]);
    CE(cec_plan_destroy(ep));
    CE(cec_plan_destroy(dp));
    CE(cec_arenas_free(slab));
    free(ev);
    free(ext);
    free(h);
    free(got);
    free(want);
    free(matrix);
    return bad ? 2 : 0;
}
