// tools/placement_modes.hip -- does where the arenas land in HBM decide the rate, and
// does a physically contiguous allocation make it repeatable?  (not product)
//
// Per trial and mode, a fresh slab of 8 arenas at cec_arena_stride(256 MiB) is
// allocated, filled on the device, and the library's encode, rotating decode (bench.py's
// masks) and fused diff-update + install (65,536 x 4 KiB SETs, random source shard) run R
// times each; the median launch time of each is printed.  Modes, interleaved per trial:
//   malloc      hipMalloc (what cec_arenas_alloc does)
//   contiguous  hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   usage: placement_modes [TRIALS [R]]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cocytus_ec.h"
#include "reed_sol.h"

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                            \
        }                                                                        \
    } while (0)
#define CE(x)                                                                    \
    do {                                                                         \
        if ((x) < 0) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, cec_last_error());                  \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__global__ void fill(uint4 *p, size_t n16, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = make_uint4((uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)(z >> 7));
    }
}

enum { K = 3, M = 2, NA = 8 };
static const size_t n = 4096, B = 65536, L = n * B;

static float median(std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 4, R = argc > 2 ? atoi(argv[2]) : 9;
    CE(cec_device_check());
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *mat = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    const size_t stride = cec_arena_stride(L);
    std::vector<cec_extent> ext(B);
    for (size_t i = 0; i < B; ++i) ext[i] = cec_extent{i * n, 0, (uint32_t)n, 0};
    cec_plan *ep, *dp, *up;
    CE(cec_plan_create(&ep, ext.data(), (int)B, s));
    uint32_t masks[K * M];
    for (int q = 0; q < M; ++q)
        for (int j = 0; j < K; ++j) {
            int conn[K + M];
            for (int i = 0; i < K + M; ++i) conn[i] = i != j;
            masks[q * K + j] = cec_recovery_mask(K, M, K + q, conn);
        }
    for (size_t i = 0; i < B; ++i) ext[i].pattern = (uint32_t)(i % (K * M));
    CE(cec_plan_create(&dp, ext.data(), (int)B, s));
    uint64_t x = 12345;
    for (size_t i = 0; i < B; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        ext[i] = cec_extent{i * n, i * n, (uint32_t)n, (uint32_t)((x >> 33) % K)};
    }
    CE(cec_plan_create(&up, ext.data(), (int)B, s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[2] = {"malloc", "contiguous"};
    for (int t = 0; t < T; ++t)
        for (int mode = 0; mode < 2; ++mode) {
            uint8_t *slab = nullptr;
            hipError_t ae = mode == 0 ? hipMalloc(&slab, stride * NA)
                                      : hipExtMallocWithFlags((void **)&slab, stride * NA, hipDeviceMallocContiguous);
            if (ae != hipSuccess) {
                (void)hipGetLastError();
                printf("{\"trial\": %d, \"mode\": \"%s\", \"error\": \"%s\"}\n", t, names[mode], hipGetErrorString(ae));
                fflush(stdout);
                continue;
            }
            uint8_t *ar[NA];
            for (int i = 0; i < NA; ++i) ar[i] = slab + i * stride;
            fill<<<4096, 256, 0, s>>>((uint4 *)slab, stride * NA / 16, 77 + t);
            const uint8_t *data[K] = {ar[0], ar[1], ar[2]};
            uint8_t *par[M] = {ar[3], ar[4]}, *out[K] = {ar[5], ar[6], ar[7]}, *dat[K] = {ar[0], ar[1], ar[2]};
            const uint8_t *surv[K + M] = {ar[0], ar[1], ar[2], ar[3], ar[4]};
            std::vector<float> te, td, tu;
            for (int r = 0; r < R + 1; ++r) {
                float ms;
                CK(hipEventRecord(e0, s));
                CE(cec_encode(K, M, mat, data, par, ep, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) te.push_back(ms * 1e3f);
                CK(hipEventRecord(e0, s));
                CE(cec_decode(K, M, mat, masks, K * M, surv, out, dp, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) td.push_back(ms * 1e3f);
                CK(hipEventRecord(e0, s));
                CE(cec_diff_update(K, M, mat, dat, ar[5 + (r & 1)], par, 1, up, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) tu.push_back(ms * 1e3f);
            }
            const float me = median(te), md = median(td), mu = median(tu);
            printf("{\"trial\": %d, \"mode\": \"%s\", \"encode_us\": %.1f, \"encode_TBps\": %.3f, \"decode_us\": %.1f, "
                   "\"decode_TBps\": %.3f, \"diff_update_us\": %.1f, \"diff_update_TBps\": %.3f}\n",
                   t, names[mode], me, 5.0 * L / me / 1e6, md, 4.0 * L / md / 1e6, mu, 7.0 * L / mu / 1e6);
            fflush(stdout);
            CK(hipFree(slab));
        }
    cec_plan_destroy(ep);
    cec_plan_destroy(dp);
    cec_plan_destroy(up);
    return 0;
}
