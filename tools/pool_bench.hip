// tools/pool_bench.hip -- the idle recoverer's traffic through cec_recovery_pool, driven from
// native code so the host loop is not Python (not product).
//
// RS(3,2), D0 lost, leader P0.  N single-unit requests (do_recovery(NULL, s, s),
// memcached.c:5712-5734) in windows of W: begin W requests, the two data peers' replies
// (4 KiB each, from pageable host memory, or written straight into the pool's staging =
// "received in place"), one flush, one batched solve into the lost lid's arena in HBM,
// end.  W = 85 is TOO_MANY_RECOVERY (const.h:27).  The same units through one
// cec_recovery session per request are timed on a prefix for comparison.  The rebuilt
// arena is checked against D0.  Prints one JSON line per configuration.
//   make -C tools   (needs cocytus_amd/libcocytus_ec.so)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/cocytus_ec.h"
#include "../include/reed_sol.h"

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            exit(1);                                                        \
        }                                                                   \
    } while (0)
#define CE(x)                                                               \
    do {                                                                    \
        int r_ = (x);                                                       \
        if (r_ < 0) {                                                       \
            fprintf(stderr, "%s: %d %s\n", #x, r_, cec_last_error());       \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 65536;  // units (4 KiB each)
    const int k = 3, m = 2;
    const size_t U = 4096, L = static_cast<size_t>(N) * U;
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(k + m, k, 8);
    CK(hipSetDevice(0));
    // host data shards (pageable: what the peers' replies hold)
    std::vector<std::vector<uint8_t>> D(k, std::vector<uint8_t>(L));
    uint64_t x = 0xC0C70A11ull;
    for (int j = 0; j < k; ++j)
        for (size_t i = 0; i < L; i += 8) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            memcpy(&D[j][i], &z, 8);
        }
    // device arenas: D0..D2 (to encode), P0, P1, rebuilt D0
    uint8_t *ar[6];
    void *slab;
    CE(cec_arenas_alloc(6, L, ar, &slab));
    for (int j = 0; j < k; ++j) CK(hipMemcpy(ar[j], D[j].data(), L, hipMemcpyHostToDevice));
    uint8_t *parity[2] = {ar[3], ar[4]};
    CE(cec_encode_region(k, m, matrix, ar, parity, L, nullptr));
    CK(hipDeviceSynchronize());
    uint8_t *out = ar[5];
    uint8_t *outs[3] = {out, nullptr, nullptr};
    const int connected[5] = {0, 1, 1, 1, 1};
    const uint32_t mask = cec_recovery_mask(k, m, k, connected);  // {D1, D2, P0}
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<uint8_t> check(L);

    for (int inplace = 0; inplace < 2; ++inplace)
        for (int W : {85, 1024}) {
            CK(hipMemset(out, 0, L));
            CK(hipDeviceSynchronize());
            cec_recovery_pool *pool;
            CE(cec_recovery_pool_create(&pool, k, m, matrix, k, ar[3], W));
            std::vector<int> ids(W);
            double t0 = 0;
            for (int pass = 0; pass < 2; ++pass) {  // pass 0 warms up (first-touch of staging)
                if (pass == 1) t0 = now();
                for (int base = 0; base < N; base += W) {
                    const int w = std::min(W, N - base);
                    for (int i = 0; i < w; ++i) {
                        const int unit = base + i;
                        ids[i] = cec_recovery_pool_begin(pool, mask, unit, unit);
                        CE(ids[i]);
                        for (int peer = 1; peer < k; ++peer) {
                            const uint8_t *src = D[peer].data() + static_cast<size_t>(unit) * U;
                            if (inplace) {  // recv straight into the pool's staging
                                size_t n;
                                uint8_t *dst = cec_recovery_pool_staging(pool, ids[i], peer, &n);
                                memcpy(dst, src, n);
                                CE(cec_recovery_pool_add_peer(pool, ids[i], peer, dst));
                            } else {
                                CE(cec_recovery_pool_add_peer(pool, ids[i], peer, src));
                            }
                        }
                    }
                    CE(cec_recovery_pool_flush_solve(pool, outs, s));  // fold + solve: one launch
                    for (int i = 0; i < w; ++i) CE(cec_recovery_pool_end(pool, ids[i]));
                }
            }
            const double t = now() - t0;
            CE(cec_recovery_pool_destroy(pool));
            CK(hipMemcpy(check.data(), out, L, hipMemcpyDeviceToHost));
            const bool ok = memcmp(check.data(), D[0].data(), L) == 0;
            printf("{\"path\": \"pool\", \"replies\": \"%s\", \"window\": %d, \"units\": %d, \"ms\": %.3f, "
                   "\"GiBps\": %.3f, \"us_per_unit\": %.3f, \"verified\": %s}\n",
                   inplace ? "received into the pool's pinned staging" : "pageable host buffers (copied)", W, N,
                   t * 1e3, L / t / (1 << 30), t * 1e6 / N, ok ? "true" : "false");
            fflush(stdout);
        }

    // one cec_recovery session per single-unit request (prefix of the range)
    const int NS = std::min(N, 4096);
    CK(hipMemset(out, 0, L));
    double t0 = 0;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) t0 = now();
        for (int unit = 0; unit < NS; ++unit) {
            cec_recovery *r;
            CE(cec_recovery_create(&r, k, m, matrix, k, mask, unit, unit, ar[3], s));
            CE(cec_recovery_add_peer(r, 1, D[1].data() + static_cast<size_t>(unit) * U, s));
            void *o[3] = {out + static_cast<size_t>(unit) * U, nullptr, nullptr};  // the unit's bytes
            CE(cec_recovery_finish(r, 2, D[2].data() + static_cast<size_t>(unit) * U, nullptr, o, s));
            CE(cec_recovery_destroy(r));
        }
    }
    const double t = now() - t0;
    CK(hipMemcpy(check.data(), out, static_cast<size_t>(NS) * U, hipMemcpyDeviceToHost));
    const bool ok = memcmp(check.data(), D[0].data(), static_cast<size_t>(NS) * U) == 0;
    printf("{\"path\": \"session per request\", \"replies\": \"pageable host buffers\", \"units\": %d, "
           "\"ms\": %.3f, \"GiBps\": %.3f, \"us_per_unit\": %.3f, \"verified\": %s}\n",
           NS, t * 1e3, NS * U / t / (1 << 30), t * 1e6 / NS, ok ? "true" : "false");
    CE(cec_arenas_free(slab));
    free(matrix);
    return 0;
}
