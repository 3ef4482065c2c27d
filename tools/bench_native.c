/*
 * tools/bench_native.c -- bench.py's metric step driven through the C-ABI alone: a C99
 * program with no HIP header, no Python and no torch, linked -lcocytus_ec.  It shows
 * the library is the product and torch only plumbing (not product; a cross-check).
 *
 * RS(3,2), 65,536 stripes of 4 KiB per GPU in arenas from cec_arenas_alloc (odd-4 KiB
 * stride), data filled from the host with splitmix64 bytes (cec_copy), one encode + one
 * decode per step, the lost data shard and the leader rotating over all (lost, leader)
 * pairs as in bench.py (masks from cec_recovery_mask = start_recovery,
 * memcached.c:8136-8151), one event between consecutive launches, W warm-up steps then S
 * timed steps.  Every rebuilt shard is compared with its original.  Prints one JSON line.
 *
 * Multi-GPU: G host threads, one per GPU, each with its own stream and its
 * own batch (no collective); a barrier before and after the timed steps; the time is the
 * max over threads and the value all threads' payload over it.  CEC_NATIVE_DEVICE=d puts
 * every thread on device d (a one-card rehearsal of the threaded path).
 * CEC_NATIVE_STRIPES=b runs b stripes per GPU instead of 65,536: the per-GPU share of
 * the strong-scaling split (8,192 at 8 GPUs), timed with no Python in the loop.
 *   usage: bench_native [S [W [G]]]        make -C tools   (needs cocytus_amd/libcocytus_ec.so)
 */
#include <cocytus_ec.h>
#include <reed_sol.h>

#include <pthread.h>
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
            a->rc = 1;                                                      \
            goto done;                                                      \
        }                                                                   \
    } while (0)

enum { K = 3, M = 2, NMASK = K * M };
static const size_t n = 4096;
static size_t B = 65536; /* stripes per GPU; CEC_NATIVE_STRIPES: one GPU's share of a fixed batch */

typedef struct {
    int device, S, W, rc;
    double elapsed, enc_ms, dec_ms;
    size_t bad;
    pthread_barrier_t *bar;
} worker_arg;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void *worker(void *p) {
    worker_arg *a = (worker_arg *)p;
    const size_t L = n * B;
    const int S = a->S, W = a->W;
    int *matrix = NULL;
    void *slab = NULL, *stream = NULL, **ev = NULL;
    uint8_t *h = NULL, *got = NULL, *want = NULL;
    cec_extent *ext = NULL;
    cec_plan *ep = NULL, *dp = NULL;
    int waited = 0;
    uint8_t *ar[K + M + K];
    uint32_t masks[NMASK];
    int lost_of[NMASK];
    CE(cec_set_device(a->device));
    CE(cec_stream_create(&stream));
    matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    if (!matrix) {
        a->rc = 1;
        goto done;
    }
    CE(cec_arenas_alloc(K + M + K, L, ar, &slab));
    uint8_t *data[K] = {ar[0], ar[1], ar[2]}, *parity[M] = {ar[3], ar[4]};
    uint8_t *out[K] = {ar[5], ar[6], ar[7]};
    const uint8_t *survivors[K + M] = {ar[0], ar[1], ar[2], ar[3], ar[4]};
    h = malloc(L);
    uint64_t x = 0xC0C70002ull + 0x100ull * (uint64_t)a->device;
    for (int j = 0; j < K; ++j) {
        for (size_t i = 0; i < L; i += 8) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            memcpy(h + i, &z, 8);
        }
        CE(cec_copy(data[j], h, L, stream));
        CE(cec_stream_synchronize(stream));
    }
    for (int q = 0; q < M; ++q)
        for (int j = 0; j < K; ++j) {
            int conn[K + M];
            for (int i = 0; i < K + M; ++i) conn[i] = i != j;
            masks[q * K + j] = cec_recovery_mask(K, M, K + q, conn);
            lost_of[q * K + j] = j;
        }
    ext = malloc(sizeof(cec_extent) * B);
    for (size_t s = 0; s < B; ++s) {
        ext[s].off = s * n;
        ext[s].src_off = 0;
        ext[s].len = (uint32_t)n;
        ext[s].pattern = 0;
    }
    CE(cec_plan_create(&ep, ext, (int)B, stream));
    for (size_t s = 0; s < B; ++s) ext[s].pattern = (uint32_t)(s % NMASK);
    CE(cec_plan_create(&dp, ext, (int)B, stream));
    for (int w = 0; w < W; ++w) {
        CE(cec_encode(K, M, matrix, (const uint8_t *const *)data, parity, ep, stream));
        CE(cec_decode(K, M, matrix, masks, NMASK, survivors, out, dp, stream));
    }
    CE(cec_stream_synchronize(stream));
    ev = calloc((size_t)(2 * S + 1), sizeof(void *));
    for (int i = 0; i < 2 * S + 1; ++i) CE(cec_event_create(&ev[i]));

    pthread_barrier_wait(a->bar);  /* every GPU ready: start together */
    waited = 1;
    const double t0 = now();
    CE(cec_event_record(ev[0], stream));
    for (int s = 0; s < S; ++s) {
        CE(cec_encode(K, M, matrix, (const uint8_t *const *)data, parity, ep, stream));
        CE(cec_event_record(ev[2 * s + 1], stream));
        CE(cec_decode(K, M, matrix, masks, NMASK, survivors, out, dp, stream));
        CE(cec_event_record(ev[2 * s + 2], stream));
    }
    CE(cec_stream_synchronize(stream));
    a->elapsed = now() - t0;
    pthread_barrier_wait(a->bar);
    waited = 2;
    for (int s = 0; s < S; ++s) {
        float e1, e2;
        CE(cec_event_elapsed_ms(ev[2 * s], ev[2 * s + 1], &e1));
        CE(cec_event_elapsed_ms(ev[2 * s + 1], ev[2 * s + 2], &e2));
        a->enc_ms += e1 / S;
        a->dec_ms += e2 / S;
    }
    /* verify: every stripe's rebuilt shard equals the original */
    got = malloc(L);
    want = malloc(L);
    for (int j = 0; j < K; ++j) {
        CE(cec_copy(got, out[j], L, stream));
        CE(cec_copy(want, data[j], L, stream));
        CE(cec_stream_synchronize(stream));
        for (size_t s = 0; s < B; ++s)
            if (lost_of[s % NMASK] == j && memcmp(got + s * n, want + s * n, n) != 0) ++a->bad;
    }
done:
    /* a failed thread still meets the barriers the others wait at */
    if (waited < 1) pthread_barrier_wait(a->bar);
    if (waited < 2) pthread_barrier_wait(a->bar);
    if (ev)
        for (int i = 0; i < 2 * S + 1; ++i)
            if (ev[i]) cec_event_destroy(ev[i]);
    if (ep) cec_plan_destroy(ep);
    if (dp) cec_plan_destroy(dp);
    if (slab) cec_arenas_free(slab);
    if (stream) cec_stream_destroy(stream);
    free(ev);
    free(ext);
    free(h);
    free(got);
    free(want);
    free(matrix);
    return NULL;
}

int main(int argc, char **argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 20, W = argc > 2 ? atoi(argv[2]) : 3;
    int G = argc > 3 ? atoi(argv[3]) : 1, ndev = 0;
    const char *pin = getenv("CEC_NATIVE_DEVICE");
    const char *stripes = getenv("CEC_NATIVE_STRIPES");
    if (stripes && *stripes) B = (size_t)strtoull(stripes, NULL, 0);
    if (B < NMASK || B > 65536) {
        fprintf(stderr, "CEC_NATIVE_STRIPES = %zu outside [%d, 65536]\n", B, NMASK);
        return 1;
    }
    if (cec_device_count(&ndev) != CEC_OK || ndev < 1 || cec_device_check() != CEC_OK) {
        fprintf(stderr, "no usable gfx950 device: %s\n", cec_last_error());
        return 1;
    }
    if (G < 1 || (!pin && G > ndev)) {
        fprintf(stderr, "G = %d threads but %d devices (CEC_NATIVE_DEVICE pins all to one)\n", G, ndev);
        return 1;
    }
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)G);
    worker_arg *args = calloc((size_t)G, sizeof(worker_arg));
    pthread_t *tid = calloc((size_t)G, sizeof(pthread_t));
    for (int g = 0; g < G; ++g) {
        args[g].device = pin ? atoi(pin) : g;
        args[g].S = S;
        args[g].W = W;
        args[g].bar = &bar;
        pthread_create(&tid[g], NULL, worker, &args[g]);
    }
    double el = 0, enc = 0, dec = 0;
    size_t bad = 0;
    int rc = 0;
    for (int g = 0; g < G; ++g) {
        pthread_join(tid[g], NULL);
        if (args[g].elapsed > el) el = args[g].elapsed;  /* max over GPUs */
        enc += args[g].enc_ms / G;
        dec += args[g].dec_ms / G;
        bad += args[g].bad;
        rc |= args[g].rc;
    }
    const double L = (double)(n * B);
    const double payload = (double)(K + 1) * L * S * G;
    printf("{\"metric\": \"GiB/s device-resident RS(3,2) encode+decode, 4 KiB values\", "
           "\"harness\": \"tools/bench_native.c (C-ABI only, no Python / torch; one thread per GPU)\", "
           "\"value\": %.2f, \"unit\": \"GiB/s\", \"n_gpus\": %d, \"devices\": \"%s\", \"steps\": %d, "
           "\"warmup\": %d, \"ms_per_step\": %.4f, \"encode_ms\": %.4f, \"encode_frac\": %.4f, "
           "\"decode_ms\": %.4f, \"decode_frac\": %.4f, \"stripes_per_gpu\": %zu, \"verified\": %s}\n",
           el > 0 ? payload / el / (double)(1u << 30) : 0.0, G, pin ? "one card (CEC_NATIVE_DEVICE)" : "0..G-1",
           S, W, el * 1e3 / S, enc, (double)(K + M) * L / (enc * 1e-3) / 8e12, dec,
           (double)(K + 1) * L / (dec * 1e-3) / 8e12, B, (bad || rc) ? "false" : "true");
    pthread_barrier_destroy(&bar);
    free(args);
    free(tid);
    return rc ? 1 : bad ? 2 : 0;
}
