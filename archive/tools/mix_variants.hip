// tools/mix_variants.hip -- access-shape probe for a 3-read / 2-write stream (the RS(3,2)
// encode mix), XOR compute, random bytes, arenas at the odd-4 KiB stride of
// cec_arenas_alloc.  Variants: workgroup size, bytes per workgroup, XCD-aware
// block -> tile remap, store policy.  Not product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mix_variants.hip -o tools/mix_variants.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GL __attribute__((address_space(1)))

struct P5 {
    const uint8_t *r0, *r1, *r2;
    uint8_t *w0, *w1;
};

__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__device__ inline u32x4 ldn(const uint8_t *p, uint64_t o) {
    return __builtin_nontemporal_load((const GL u32x4 *)((uintptr_t)p + o));
}
template <bool NT>
__device__ inline void stn(uint8_t *p, uint64_t o, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)p + o));
    else *(GL u32x4 *)((uintptr_t)p + o) = v;
}

// BLOCK threads, CH chunks of 16 B per lane (lane-strided by BLOCK*16), one
// BLOCK*16*CH-byte tile per workgroup.  XCD: remap block b so XCD (b % 8) walks a
// contiguous eighth of the arena.
template <int BLOCK, int CH, bool XCD, bool NT>
__global__ __launch_bounds__(BLOCK) void k_v(P5 p, uint32_t ntiles) {
    uint32_t b = blockIdx.x;
    if constexpr (XCD) {
        const uint32_t per = ntiles / 8;
        b = (b % 8) * per + b / 8;
    }
    const uint64_t base = (uint64_t)b * (BLOCK * 16 * CH) + threadIdx.x * 16;
    u32x4 a[CH], c[CH], d[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) {
        const uint64_t o = base + q * BLOCK * 16;
        a[q] = ldn(p.r0, o);
        c[q] = ldn(p.r1, o);
        d[q] = ldn(p.r2, o);
    }
#pragma unroll
    for (int q = 0; q < CH; ++q) {
        const uint64_t o = base + q * BLOCK * 16;
        u32x4 x = a[q] ^ c[q] ^ d[q];
        stn<NT>(p.w0, o, x);
        x.x ^= 0x1D;
        stn<NT>(p.w1, o, x);
    }
}

// CombineArgs-like kernarg: 48 base pointers selected by per-launch stream ids.
struct Big {
    uint8_t *base[48];
    int ids[8];
};
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_big(Big a) {
    const uint64_t o = (uint64_t)blockIdx.x * (BLOCK * 16) + threadIdx.x * 16;
    const u32x4 x0 = ldn(a.base[a.ids[0]], o), x1 = ldn(a.base[a.ids[1]], o), x2 = ldn(a.base[a.ids[2]], o);
    u32x4 x = x0 ^ x1 ^ x2;
    stn<true>(a.base[a.ids[3]], o, x);
    x.x ^= 0x1D;
    stn<true>(a.base[a.ids[4]], o, x);
}
// the same block read from ordinary (cacheable) device memory through one pointer
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_ind(const Big *ap) {
    const __attribute__((address_space(4))) Big *a = (const __attribute__((address_space(4))) Big *)(uintptr_t)ap;
    const uint64_t o = (uint64_t)blockIdx.x * (BLOCK * 16) + threadIdx.x * 16;
    const u32x4 x0 = ldn(a->base[a->ids[0]], o), x1 = ldn(a->base[a->ids[1]], o), x2 = ldn(a->base[a->ids[2]], o);
    u32x4 x = x0 ^ x1 ^ x2;
    stn<true>(a->base[a->ids[3]], o, x);
    x.x ^= 0x1D;
    stn<true>(a->base[a->ids[4]], o, x);
}

int main() {
    const uint64_t L = 256ull << 20;
    const uint64_t stride = L + 4096;  // cec_arena_stride(L)
    uint8_t *slab;
    CK(hipMalloc(&slab, 5 * stride));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_fill, 4096, 256, 0, 0, (uint64_t *)(slab + i * stride), L / 8, 77ull + i);
    CK(hipDeviceSynchronize());
    P5 p{slab, slab + stride, slab + 2 * stride, slab + 3 * stride, slab + 4 * stride};
    Big big{};
    for (int i = 0; i < 48; ++i) big.base[i] = slab + (i % 5) * stride;
    for (int i = 0; i < 5; ++i) big.ids[i] = 5 * (i + 2) + i;  // base[id] is arena id % 5 = i
    Big *dbig;
    CK(hipMalloc(&dbig, sizeof(Big)));
    CK(hipMemcpy(dbig, &big, sizeof(Big), hipMemcpyHostToDevice));
    struct V {
        const char *name;
        int id;
    };
    std::vector<V> vs = {
        {"256 thr x 1 chunk (4 KiB/WG) nt   [product]", 0},
        {"256 thr x 2 chunks (8 KiB/WG) nt", 1},
        {"256 thr x 4 chunks (16 KiB/WG) nt", 2},
        {"512 thr x 1 chunk (8 KiB/WG) nt", 3},
        {"1024 thr x 1 chunk (16 KiB/WG) nt", 4},
        {"128 thr x 2 chunks (4 KiB/WG) nt", 5},
        {"64 thr x 4 chunks (4 KiB/WG) nt", 6},
        {"256 thr x 1 chunk, XCD remap nt", 7},
        {"256 thr x 1 chunk, plain stores", 8},
        {"128 thr x 1 chunk (2 KiB/WG) nt", 9},
        {"64 thr x 1 chunk (1 KiB/WG) nt", 10},
        {"64 thr x 2 chunks (2 KiB/WG) nt", 11},
        {"128 thr x 1 chunk (2 KiB/WG) plain", 12},
        {"192 thr x 1 chunk (3 KiB/WG) nt", 13},
        {"64 thr, 400-B kernarg, dynamic base index", 14},
        {"64 thr, args in device memory (1 ptr kernarg)", 15},
        {"256 thr, 400-B kernarg, dynamic base index", 16},
        {"256 thr, args in device memory", 17},
    };
    auto launch = [&](int id) {
        const uint32_t t4 = L / 4096;
        switch (id) {
        case 0: hipLaunchKernelGGL((k_v<256, 1, false, true>), t4, 256, 0, 0, p, t4); break;
        case 1: hipLaunchKernelGGL((k_v<256, 2, false, true>), t4 / 2, 256, 0, 0, p, t4 / 2); break;
        case 2: hipLaunchKernelGGL((k_v<256, 4, false, true>), t4 / 4, 256, 0, 0, p, t4 / 4); break;
        case 3: hipLaunchKernelGGL((k_v<512, 1, false, true>), t4 / 2, 512, 0, 0, p, t4 / 2); break;
        case 4: hipLaunchKernelGGL((k_v<1024, 1, false, true>), t4 / 4, 1024, 0, 0, p, t4 / 4); break;
        case 5: hipLaunchKernelGGL((k_v<128, 2, false, true>), t4, 128, 0, 0, p, t4); break;
        case 6: hipLaunchKernelGGL((k_v<64, 4, false, true>), t4, 64, 0, 0, p, t4); break;
        case 7: hipLaunchKernelGGL((k_v<256, 1, true, true>), t4, 256, 0, 0, p, t4); break;
        case 8: hipLaunchKernelGGL((k_v<256, 1, false, false>), t4, 256, 0, 0, p, t4); break;
        case 9: hipLaunchKernelGGL((k_v<128, 1, false, true>), t4 * 2, 128, 0, 0, p, t4 * 2); break;
        case 10: hipLaunchKernelGGL((k_v<64, 1, false, true>), t4 * 4, 64, 0, 0, p, t4 * 4); break;
        case 11: hipLaunchKernelGGL((k_v<64, 2, false, true>), t4 * 2, 64, 0, 0, p, t4 * 2); break;
        case 12: hipLaunchKernelGGL((k_v<128, 1, false, false>), t4 * 2, 128, 0, 0, p, t4 * 2); break;
        case 14: hipLaunchKernelGGL((k_big<64>), t4 * 4, 64, 0, 0, big); break;
        case 15: hipLaunchKernelGGL((k_ind<64>), t4 * 4, 64, 0, 0, (const Big *)dbig); break;
        case 16: hipLaunchKernelGGL((k_big<256>), t4, 256, 0, 0, big); break;
        case 17: hipLaunchKernelGGL((k_ind<256>), t4, 256, 0, 0, (const Big *)dbig); break;
        case 13: hipLaunchKernelGGL((k_v<192, 1, false, true>), (uint32_t)(L / 3072), 192, 0, 0, p, (uint32_t)(L / 3072)); break;
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 9, iters = 10;
    std::vector<std::vector<float>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            launch(vs[i].id);
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; ++it) launch(vs[i].id);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t / iters);
        }
    printf("3R:2W stream, 256 MiB per arena, odd-4KiB arena stride, random bytes\n");
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(ms[i].begin(), ms[i].end());
        printf("%-44s median %.4f ms -> %.0f GB/s (best %.0f)\n", vs[i].name, ms[i][rounds / 2],
               5.0 * L / (ms[i][rounds / 2] * 1e6), 5.0 * L / (ms[i][0] * 1e6));
    }
    return 0;
}
