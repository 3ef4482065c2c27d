// tools/encode_variants.hip -- design-space probe for the RS(K,M) encode kernel
// (not part of the product).  RS(3,2), 4 KiB values, 65,536 stripes, arenas
// contiguous; every variant computes the same parity and is checked against
// variant 0.  Timed with hipEvents, variants interleaved over rounds (one process).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/encode_variants.hip -o /tmp/ev
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../cocytus_amd/csrc/gf256.hpp"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GL __attribute__((address_space(1)))

struct Tabs {
    uint32_t t[2][3][5];  // [parity][shard][perm table]
    int coef[2][3];
};

__device__ inline uint32_t pmul(uint32_t x, const uint32_t *t) {
    const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^
           __builtin_amdgcn_perm(t[4], t[4], s2);
}

template <bool NT>
__device__ inline u32x4 ld(const uint8_t *p, uint64_t off) {
    const GL u32x4 *a = (const GL u32x4 *)((uintptr_t)p + off);
    if constexpr (NT) return __builtin_nontemporal_load(a);
    else return *a;
}
template <bool NT>
__device__ inline void st(uint8_t *p, uint64_t off, u32x4 v) {
    GL u32x4 *a = (GL u32x4 *)((uintptr_t)p + off);
    if constexpr (NT) __builtin_nontemporal_store(v, a);
    else *a = v;
}

// generic RS(3,2) combine of one 16 B chunk: row0 = all ones (XOR), row1 = tables
__device__ inline void combine(const u32x4 &a, const u32x4 &b, const u32x4 &c, const Tabs &T,
                               u32x4 &p0, u32x4 &p1, bool xor_only) {
    p0 = a ^ b ^ c;
    if (xor_only) {
        p1 = p0;
        return;
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t v = a[w];  // coef[1][0] == 1
        v ^= pmul(b[w], T.t[1][1]);
        v ^= pmul(c[w], T.t[1][2]);
        p1[w] = v;
    }
}

// V0/V1: one 4 KiB tile per block iteration, grid-stride (grid = param)
template <bool NTL, bool NTS, bool XOR_ONLY>
__global__ __launch_bounds__(256) void k_tile(const uint8_t *d0, const uint8_t *d1, const uint8_t *d2,
                                              uint8_t *p0, uint8_t *p1, uint32_t ntiles, Tabs T) {
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t off = (uint64_t)t * 4096 + threadIdx.x * 16;
        u32x4 a = ld<NTL>(d0, off), b = ld<NTL>(d1, off), c = ld<NTL>(d2, off);
        u32x4 x, y;
        combine(a, b, c, T, x, y, XOR_ONLY);
        st<NTS>(p0, off, x);
        st<NTS>(p1, off, y);
    }
}

// V2: U tiles per iteration (loads of all U issued before any compute)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_unroll(const uint8_t *d0, const uint8_t *d1, const uint8_t *d2,
                                                uint8_t *p0, uint8_t *p1, uint32_t ntiles, Tabs T) {
    for (uint32_t t = blockIdx.x * U; t < ntiles; t += gridDim.x * U) {
        u32x4 a[U], b[U], c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t off = (uint64_t)(t + u) * 4096 + threadIdx.x * 16;
            if (t + u < ntiles) {
                a[u] = ld<NTL>(d0, off);
                b[u] = ld<NTL>(d1, off);
                c[u] = ld<NTL>(d2, off);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (t + u >= ntiles) continue;
            const uint64_t off = (uint64_t)(t + u) * 4096 + threadIdx.x * 16;
            u32x4 x, y;
            combine(a[u], b[u], c[u], T, x, y, false);
            st<NTS>(p0, off, x);
            st<NTS>(p1, off, y);
        }
    }
}

// V3: software-pipelined: loads of tile t+stride issued before compute of tile t
template <bool NTS>
__global__ __launch_bounds__(256) void k_pipe(const uint8_t *d0, const uint8_t *d1, const uint8_t *d2,
                                              uint8_t *p0, uint8_t *p1, uint32_t ntiles, Tabs T) {
    uint32_t t = blockIdx.x;
    if (t >= ntiles) return;
    uint64_t off = (uint64_t)t * 4096 + threadIdx.x * 16;
    u32x4 a = ld<false>(d0, off), b = ld<false>(d1, off), c = ld<false>(d2, off);
    for (;;) {
        const uint32_t tn = t + gridDim.x;
        const uint64_t offn = (uint64_t)tn * 4096 + threadIdx.x * 16;
        u32x4 an, bn, cn;
        const bool more = tn < ntiles;
        if (more) {
            an = ld<false>(d0, offn);
            bn = ld<false>(d1, offn);
            cn = ld<false>(d2, offn);
        }
        u32x4 x, y;
        combine(a, b, c, T, x, y, false);
        st<NTS>(p0, off, x);
        st<NTS>(p1, off, y);
        if (!more) break;
        a = an; b = bn; c = cn; t = tn; off = offn;
    }
}

// V4: each thread owns 64 contiguous bytes (4 x dwordx4) of a 16 KiB block-chunk
__global__ __launch_bounds__(256) void k_wide(const uint8_t *d0, const uint8_t *d1, const uint8_t *d2,
                                              uint8_t *p0, uint8_t *p1, uint64_t len, Tabs T) {
    const uint64_t chunk = 256 * 64;
    for (uint64_t base = (uint64_t)blockIdx.x * chunk; base < len; base += (uint64_t)gridDim.x * chunk) {
        u32x4 a[4], b[4], c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t off = base + q * 4096 + threadIdx.x * 16;
            a[q] = ld<false>(d0, off);
            b[q] = ld<false>(d1, off);
            c[q] = ld<false>(d2, off);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t off = base + q * 4096 + threadIdx.x * 16;
            u32x4 x, y;
            combine(a[q], b[q], c[q], T, x, y, false);
            st<true>(p0, off, x);
            st<true>(p1, off, y);
        }
    }
}

// memory ceilings: read 3 streams + write 2 (XOR), pure copy 1->1
__global__ __launch_bounds__(256) void k_copy(const uint8_t *s, uint8_t *d, uint64_t len) {
    for (uint64_t off = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; off < len;
         off += (uint64_t)gridDim.x * 256 * 16)
        st<false>(d, off, ld<false>(s, off));
}

int main(int argc, char **argv) {
    const int K = 3, M = 2, n = 4096, B = argc > 1 ? atoi(argv[1]) : 65536;
    const uint64_t len = (uint64_t)n * B;
    int cus = 256;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    uint8_t *d[3], *p[2], *ref[2];
    for (int j = 0; j < K; ++j) CK(hipMalloc(&d[j], len));
    for (int q = 0; q < M; ++q) {
        CK(hipMalloc(&p[q], len));
        CK(hipMalloc(&ref[q], len));
    }
    std::vector<uint8_t> h(len);
    uint64_t x = 0xC0C70002;
    for (int j = 0; j < K; ++j) {
        for (uint64_t i = 0; i < len; i += 8) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            memcpy(&h[i], &z, 8);
        }
        CK(hipMemcpy(d[j], h.data(), len, hipMemcpyHostToDevice));
    }
    Tabs T;
    const int mat[2][3] = {{1, 1, 1}, {1, 245, 244}};
    for (int q = 0; q < 2; ++q)
        for (int j = 0; j < 3; ++j) {
            auto pt = cec::make_perm_tab(mat[q][j]);
            memcpy(T.t[q][j], pt.w, sizeof pt.w);
            T.coef[q][j] = mat[q][j];
        }
    const uint32_t ntiles = B;
    struct V {
        const char *name;
        int kind;
        int grid;
    };
    const int nt = (int)ntiles;
    std::vector<V> vs = {
        {"tile g=cus*8", 0, cus * 8},
        {"tile g=ntiles", 0, nt},
        {"tile ntstore g=ntiles", 1, nt},
        {"tile ntload+ntstore g=ntiles", 2, nt},
        {"unroll2 g=ntiles/2", 3, nt / 2},
        {"unroll2 ntstore g=ntiles/2", 4, nt / 2},
        {"unroll4 ntstore g=ntiles/4", 5, nt / 4},
        {"unroll2 ntstore g=ntiles/4", 4, nt / 4},
        {"tile ntstore g=ntiles/2", 1, nt / 2},
        {"tile ntstore g=ntiles/4", 1, nt / 4},
        {"wide64B ntstore g=ntiles/4", 8, nt / 4},
        {"xor-only (ceiling) g=ntiles", 9, nt},
        {"xor-only ntstore (ceiling) g=ntiles", 11, nt},
        {"copy 1->1 (ceiling) g=len/4K", 10, nt},
        {"copy 1->1 (ceiling) g=cus*8", 10, cus * 8},
    };
    auto launch = [&](const V &v) {
        dim3 g(v.grid), b(256);
        switch (v.kind) {
        case 0: hipLaunchKernelGGL((k_tile<false, false, false>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 1: hipLaunchKernelGGL((k_tile<false, true, false>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 2: hipLaunchKernelGGL((k_tile<true, true, false>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 3: hipLaunchKernelGGL((k_unroll<2, false, false>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 4: hipLaunchKernelGGL((k_unroll<2, false, true>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 5: hipLaunchKernelGGL((k_unroll<4, false, true>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 6: hipLaunchKernelGGL((k_pipe<false>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 7: hipLaunchKernelGGL((k_pipe<true>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 8: hipLaunchKernelGGL(k_wide, g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], len, T); break;
        case 9: hipLaunchKernelGGL((k_tile<false, false, true>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        case 10: hipLaunchKernelGGL(k_copy, g, b, 0, 0, d[0], p[0], len); break;
        case 11: hipLaunchKernelGGL((k_tile<false, true, true>), g, b, 0, 0, d[0], d[1], d[2], p[0], p[1], ntiles, T); break;
        }
    };
    // reference output
    launch(vs[0]);
    CK(hipDeviceSynchronize());
    for (int q = 0; q < M; ++q) CK(hipMemcpy(ref[q], p[q], len, hipMemcpyDeviceToDevice));
    std::vector<uint8_t> a(len), bb(len);
    for (size_t i = 0; i < vs.size(); ++i) {
        if (vs[i].kind >= 9) continue;
        CK(hipMemset(p[0], 0, len));
        CK(hipMemset(p[1], 0, len));
        launch(vs[i]);
        CK(hipDeviceSynchronize());
        for (int q = 0; q < M; ++q) {
            CK(hipMemcpy(a.data(), p[q], len, hipMemcpyDeviceToHost));
            CK(hipMemcpy(bb.data(), ref[q], len, hipMemcpyDeviceToHost));
            if (memcmp(a.data(), bb.data(), len)) {
                printf("MISMATCH variant %s parity %d\n", vs[i].name, q);
                return 1;
            }
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 7, iters = 20;
    std::vector<std::vector<float>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            launch(vs[i]);
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; ++it) launch(vs[i]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t / iters);
        }
    printf("RS(3,2) encode, %d x %d B stripes, %d CUs; algorithmic bytes = 5n per stripe\n", B, n, cus);
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(ms[i].begin(), ms[i].end());
        const double bytes = vs[i].kind == 10 ? 2.0 * len : 5.0 * len;
        printf("%-32s median %.4f ms  min %.4f ms  -> %.0f GB/s (median)  %.0f GB/s (best)\n",
               vs[i].name, ms[i][rounds / 2], ms[i][0], bytes / (ms[i][rounds / 2] * 1e6),
               bytes / (ms[i][0] * 1e6));
    }
    return 0;
}
