// tools/hbm_mix.hip -- HBM ceiling per read:write mix on this MI355X (not product).
// Each kernel streams R read arenas and W write arenas of `len` bytes with the access
// shape of combine_kernel (a 4 KiB tile per 256 >> s lanes x 2^s workgroups, 16 B per
// lane, nt loads/stores), XOR-combining reads into every write; grid = tiles << s.
//   argv[1]: arena layout: 0 = separate hipMalloc per arena; "arena" = one allocation at
//            the library's odd-4 KiB stride (cec_arena_stride); N = 2 MiB + i*N skew
//   argv[2]: "const" = constant bytes instead of random
//   argv[3]: lanes per workgroup (256, 128 or 64; default 256)  The GB/s of
// each mix is the practical roofline for the op with that mix:
//   encode RS(3,2) 3:2, decode single 3:1, RS(4,2) encode 4:2, drain 2:1 (RMW).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hbm_mix.hip -o tools/hbm_mix.bin
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

struct Ptrs {
    const uint8_t *r[6];
    uint8_t *w[4];
};

template <int R, int W>
__global__ __launch_bounds__(256) void k_mix(Ptrs p, uint32_t *sink) {
    const uint64_t off = (uint64_t)blockIdx.x * blockDim.x * 16 + threadIdx.x * 16;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < R; ++i)
        acc ^= __builtin_nontemporal_load((const GL u32x4 *)((uintptr_t)p.r[i] + off));
    if constexpr (W == 0) {
        if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;  // keep the loads
    } else {
#pragma unroll
        for (int j = 0; j < W; ++j) {
            u32x4 v = acc;
            v.x ^= j;
            __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)p.w[j] + off));
        }
    }
}

// The access shapes of the ops whose streams are not independent arenas:
//   kind 0: diff-update + install, 4 reads / 3 writes, 3 of them read-modify-write
//           (D_j, P0, P1 read then written; staging read): r0 = D, r1 = staging,
//           r2 = P0, r3 = P1; writes go back to r0, r2, r3
//   kind 1: the same without install (4 reads, P0 / P1 written back)
//   kind 2: RS(3,2) decode with the lost shard rotating per 4 KiB stripe and the leader
//           every 3 stripes (the bench): reads the 2 surviving data arenas (r0..r2) and
//           parity r3 / r4, writes arena 5 + lost (the bench's arena order; round 2's
//           probe wrote 6 + lost, one arena further along the slab)
//   kind 3: RS(4,2) decode, 64 KiB stripes (16 tiles), lost shard rotating per stripe:
//           reads 3 data (r0..r3) + parity r4 / r5, writes w[lost]
//   kind 4: kind 2 with a fixed lost shard (D0) and leader (P0)
template <int KIND>
__global__ __launch_bounds__(256) void k_shape(Ptrs p, uint8_t *const *all, uint32_t tile_shift) {
    const uint64_t off = (uint64_t)blockIdx.x * blockDim.x * 16 + threadIdx.x * 16;
    const uint32_t t = blockIdx.x >> tile_shift;  // 4 KiB tile index
    u32x4 acc = {0, 0, 0, 0};
    auto ld = [&](const uint8_t *b) { return __builtin_nontemporal_load((const GL u32x4 *)((uintptr_t)b + off)); };
    auto st = [&](uint8_t *b, u32x4 v) { __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)b + off)); };
    if constexpr (KIND == 0 || KIND == 1) {
        const u32x4 d = ld(all[0]), n = ld(all[1]);
        u32x4 p0 = ld(all[2]), p1 = ld(all[3]);
        const u32x4 x = d ^ n;
        p0 ^= x;
        p1 ^= x;
        st(all[2], p0);
        st(all[3], p1);
        if constexpr (KIND == 0) st(all[0], n);
    } else if constexpr (KIND == 2 || KIND == 4) {
        const uint32_t lost = KIND == 4 ? 0 : t % 3, par = KIND == 4 ? 0 : (t / 3) % 2;
        for (int j = 0; j < 3; ++j)
            if (j != (int)lost) acc ^= ld(all[j]);
        acc ^= ld(all[3 + par]);
        st(all[5 + lost], acc);  // the bench's layout: data 0-2, parity 3-4, rebuilt 5-7
    } else {
        const uint32_t stripe = t >> 4, lost = stripe % 4, par = (stripe / 4) % 2;
        for (int j = 0; j < 4; ++j)
            if (j != (int)lost) acc ^= ld(all[j]);
        acc ^= ld(all[4 + par]);
        st(all[6 + lost], acc);
    }
}

// splitmix64 fill: the ceilings must be measured on random bytes like the bench's
__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char **argv) {
    // per arena (HBM_MIX_MB overrides: the RS(4,2) 64 KiB bench uses 1 GiB arenas)
    const uint64_t len = (getenv("HBM_MIX_MB") ? strtoull(getenv("HBM_MIX_MB"), nullptr, 0) : 256ull) << 20;
    // argv[1] = skew in bytes: arena i starts i * skew past a 2 MiB boundary inside one
    // allocation (0 = separate hipMalloc per arena, the default layout)
    const bool arena = argc > 1 && argv[1][0] == 'a';
    const uint64_t skew = argc > 1 && !arena ? strtoull(argv[1], nullptr, 0) : 0;
    const uint32_t lanes = argc > 3 ? (uint32_t)atoi(argv[3]) : 256;
    if (lanes != 256 && lanes != 128 && lanes != 64) {
        fprintf(stderr, "lanes must be 256, 128 or 64\n");
        return 1;
    }
    // argv[2] == "const": constant bytes (hipMemset) instead of random ones
    const bool constant = argc > 2 && argv[2][0] == 'c';
    auto fill = [&](uint8_t *b, int i) {
        if (constant) CK(hipMemset(b, i * 7 + 1, len));
        else hipLaunchKernelGGL(k_fill, 4096, 256, 0, 0, (uint64_t *)b, len / 8, 0xC0C70000ull + i);
        CK(hipDeviceSynchronize());
    };
    printf("fill: %s\n", constant ? "constant" : "random");
    Ptrs p;
    std::vector<uint8_t *> bufs;
    if (arena) {  // cec_arena_stride: an odd number of 4 KiB pages between bases
        uint64_t pages = (len + 4095) / 4096;
        if (pages % 2 == 0) ++pages;
        const uint64_t stride = pages * 4096;
        uint8_t *big;
        CK(hipMalloc(&big, 10 * stride));
        for (int i = 0; i < 10; ++i) {
            uint8_t *b = big + i * stride;
            fill(b, i);
            bufs.push_back(b);
        }
    } else if (skew == 0) {
        for (int i = 0; i < 10; ++i) {
            uint8_t *b;
            CK(hipMalloc(&b, len));
            fill(b, i);
            bufs.push_back(b);
        }
    } else {
        const uint64_t stride = len + (2ull << 20);
        uint8_t *big;
        CK(hipMalloc(&big, 10 * stride + 10 * skew));
        for (int i = 0; i < 10; ++i) {
            uint8_t *b = big + i * stride + i * skew;
            fill(b, i);
            bufs.push_back(b);
        }
    }
    printf("arena layout: %s, %u lanes per workgroup\n",
           arena ? "one allocation, odd-4KiB stride" : (skew ? "skewed" : "separate hipMalloc"), lanes);
    for (int i = 0; i < 6; ++i) p.r[i] = bufs[i];
    for (int j = 0; j < 4; ++j) p.w[j] = bufs[6 + j];
    uint32_t *sink;
    CK(hipMalloc(&sink, 4));
    struct V {
        const char *name;
        int r, w;
    };
    std::vector<V> vs = {{"read 1", 1, 0}, {"read 3", 3, 0}, {"write 1 (from read 0)", 0, 1},
                         {"1:1 copy", 1, 1}, {"2:1 (RMW-like)", 2, 1}, {"3:1 decode RS(3,2)", 3, 1},
                         {"3:2 encode RS(3,2)", 3, 2}, {"4:1 decode RS(4,2)", 4, 1},
                         {"4:2 encode RS(4,2)", 4, 2}, {"6:4 RS(6,4)-like", 6, 4}};
    uint8_t **all;
    CK(hipMalloc(&all, 10 * sizeof(uint8_t *)));
    CK(hipMemcpy(all, bufs.data(), 10 * sizeof(uint8_t *), hipMemcpyHostToDevice));
    uint32_t tshift = lanes == 256 ? 0 : lanes == 128 ? 1 : 2;
    struct S {
        const char *name;
        int kind, r, w;
    };
    std::vector<S> shapes = {{"diff-update+install 4:3 (3 RMW)", 0, 4, 3},
                             {"diff-update 4:2 (2 RMW)", 1, 4, 2},
                             {"RS(3,2) decode, rotating 3:1", 2, 3, 1},
                             {"RS(3,2) decode, fixed 3:1", 4, 3, 1},
                             {"RS(4,2) 64K decode, rotating 4:1", 3, 4, 1}};
    for (const S &sh : shapes) vs.push_back({sh.name, 100 + sh.kind, 0});
    const uint32_t grid = len / (16 * lanes);
    auto launch = [&](const V &v) {
        switch (v.r * 10 + v.w) {
        case 10: hipLaunchKernelGGL((k_mix<1, 0>), grid, lanes, 0, 0, p, sink); break;
        case 30: hipLaunchKernelGGL((k_mix<3, 0>), grid, lanes, 0, 0, p, sink); break;
        case 1: hipLaunchKernelGGL((k_mix<0, 1>), grid, lanes, 0, 0, p, sink); break;
        case 11: hipLaunchKernelGGL((k_mix<1, 1>), grid, lanes, 0, 0, p, sink); break;
        case 21: hipLaunchKernelGGL((k_mix<2, 1>), grid, lanes, 0, 0, p, sink); break;
        case 31: hipLaunchKernelGGL((k_mix<3, 1>), grid, lanes, 0, 0, p, sink); break;
        case 32: hipLaunchKernelGGL((k_mix<3, 2>), grid, lanes, 0, 0, p, sink); break;
        case 41: hipLaunchKernelGGL((k_mix<4, 1>), grid, lanes, 0, 0, p, sink); break;
        case 42: hipLaunchKernelGGL((k_mix<4, 2>), grid, lanes, 0, 0, p, sink); break;
        case 64: hipLaunchKernelGGL((k_mix<6, 4>), grid, lanes, 0, 0, p, sink); break;
        case 1000: hipLaunchKernelGGL((k_shape<0>), grid, lanes, 0, 0, p, all, tshift); break;
        case 1010: hipLaunchKernelGGL((k_shape<1>), grid, lanes, 0, 0, p, all, tshift); break;
        case 1020: hipLaunchKernelGGL((k_shape<2>), grid, lanes, 0, 0, p, all, tshift); break;
        case 1030: hipLaunchKernelGGL((k_shape<3>), grid, lanes, 0, 0, p, all, tshift); break;
        case 1040: hipLaunchKernelGGL((k_shape<4>), grid, lanes, 0, 0, p, all, tshift); break;
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 7, iters = 10;
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
    printf("HBM ceilings by read:write mix, %llu MiB per arena, %u B per workgroup, nt\n",
           (unsigned long long)(len >> 20), lanes * 16);
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(ms[i].begin(), ms[i].end());
        double bytes = (double)(vs[i].r + vs[i].w) * len;
        if (vs[i].r >= 100) {  // access shapes: bytes per op
            const int kind = vs[i].r - 100;
            const int rw[5] = {7, 6, 4, 5, 4};
            bytes = (double)rw[kind] * len;
        }
        printf("%-24s median %.4f ms -> %.0f GB/s (best %.0f)\n", vs[i].name, ms[i][rounds / 2],
               bytes / (ms[i][rounds / 2] * 1e6), bytes / (ms[i][0] * 1e6));
    }
    return 0;
}
