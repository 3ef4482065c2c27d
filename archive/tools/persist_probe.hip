// tools/persist_probe.hip -- why the library does not gain from an occupancy cap that
// speeds up a bare stream (tools/policy_probe.hip), and whether a persistent,
// software-pipelined walk of the tile list recovers it.  RS(3,2) encode shape:
// 3 reads + 2 writes of 1 KiB per work item (quarter 4 KiB tile), 64-lane workgroups,
// arenas at the odd-4 KiB stride.  Not product.
//   bare     : addresses from blockIdx (policy_probe's kernel)
//   meta     : a work item first loads its tile {off, pattern} and the pattern's stream
//              ids (scalar loads), like combine_kernel
//   persist  : grid = CUs x cap, each workgroup walks items g, g + grid, ... with meta
//   pipe     : persist, with the next item's metadata and stream loads issued before the
//              current item's XOR + stores (register double buffer)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/persist_probe.hip -o tools/persist_probe.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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
#define CS __attribute__((address_space(4)))

struct Tile {
    uint64_t off, src_off;
    uint32_t len, pattern;
};
struct Pat {
    int32_t in_stream[4];
    int32_t out_stream[4];
};
struct Args {
    uint8_t *base[8];
    const Tile *tiles;
    const Pat *pats;
    uint32_t n_items;  // work items = tiles x 4
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
__device__ inline void stn(uint8_t *p, uint64_t o, u32x4 v) {
    __builtin_nontemporal_store(v, (GL u32x4 *)((uintptr_t)p + o));
}

__global__ __launch_bounds__(64) void k_bare(Args a) {
    const uint64_t o = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 16;
    u32x4 x = ldn(a.base[0], o) ^ ldn(a.base[1], o) ^ ldn(a.base[2], o);
    stn(a.base[3], o, x);
    x.x ^= 0x1D;
    stn(a.base[4], o, x);
}

struct Item {
    const uint8_t *in0, *in1, *in2;
    uint8_t *o0, *o1;
};
__device__ inline Item item(const Args &a, uint32_t g) {
    const CS Tile *t = (const CS Tile *)(uintptr_t)(a.tiles) + (g >> 2);
    const uint64_t off = t->off + (g & 3) * 1024;
    const CS Pat *p = (const CS Pat *)(uintptr_t)(a.pats) + t->pattern;
    return Item{a.base[p->in_stream[0]] + off, a.base[p->in_stream[1]] + off, a.base[p->in_stream[2]] + off,
                a.base[p->out_stream[0]] + off, a.base[p->out_stream[1]] + off};
}

__global__ __launch_bounds__(64) void k_meta(Args a) {
    const Item it = item(a, blockIdx.x);
    const uint32_t l = threadIdx.x * 16;
    u32x4 x = ldn(it.in0, l) ^ ldn(it.in1, l) ^ ldn(it.in2, l);
    stn(it.o0, l, x);
    x.x ^= 0x1D;
    stn(it.o1, l, x);
}

// tile from the list, stream bases straight from the kernarg (pattern resolved on the host)
__global__ __launch_bounds__(64) void k_tile(Args a) {
    const CS Tile *t = (const CS Tile *)(uintptr_t)(a.tiles) + (blockIdx.x >> 2);
    const uint64_t o = t->off + (blockIdx.x & 3) * 1024 + threadIdx.x * 16;
    u32x4 x = ldn(a.base[0], o) ^ ldn(a.base[1], o) ^ ldn(a.base[2], o);
    stn(a.base[3], o, x);
    x.x ^= 0x1D;
    stn(a.base[4], o, x);
}

__global__ __launch_bounds__(64) void k_persist(Args a) {
    const uint32_t l = threadIdx.x * 16;
    for (uint32_t g = blockIdx.x; g < a.n_items; g += gridDim.x) {
        const Item it = item(a, g);
        u32x4 x = ldn(it.in0, l) ^ ldn(it.in1, l) ^ ldn(it.in2, l);
        stn(it.o0, l, x);
        x.x ^= 0x1D;
        stn(it.o1, l, x);
    }
}

__global__ __launch_bounds__(64) void k_pipe(Args a) {
    const uint32_t l = threadIdx.x * 16;
    uint32_t g = blockIdx.x;
    if (g >= a.n_items) return;
    Item cur = item(a, g);
    u32x4 x0 = ldn(cur.in0, l), x1 = ldn(cur.in1, l), x2 = ldn(cur.in2, l);
    for (;;) {
        const uint32_t gn = g + gridDim.x;
        const bool more = gn < a.n_items;
        Item nxt = cur;
        u32x4 y0, y1, y2;
        if (more) {
            nxt = item(a, gn);
            y0 = ldn(nxt.in0, l);
            y1 = ldn(nxt.in1, l);
            y2 = ldn(nxt.in2, l);
        }
        u32x4 x = x0 ^ x1 ^ x2;
        stn(cur.o0, l, x);
        x.x ^= 0x1D;
        stn(cur.o1, l, x);
        if (!more) break;
        cur = nxt;
        x0 = y0;
        x1 = y1;
        x2 = y2;
        g = gn;
    }
}

int main(int argc, char **argv) {
    const uint64_t L = 256ull << 20;
    const uint64_t stride = L + 4096;
    uint8_t *slab;
    CK(hipMalloc(&slab, 5 * stride));
    for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL(k_fill, 4096, 256, 0, 0, (uint64_t *)(slab + i * stride), L / 8, 77ull + i);
    const uint32_t ntiles = L / 4096;
    std::vector<Tile> ht(ntiles);
    for (uint32_t t = 0; t < ntiles; ++t) ht[t] = Tile{(uint64_t)t * 4096, 0, 4096, 0};
    Tile *dt;
    CK(hipMalloc(&dt, ntiles * sizeof(Tile)));
    CK(hipMemcpy(dt, ht.data(), ntiles * sizeof(Tile), hipMemcpyHostToDevice));
    Pat hp{{0, 1, 2, 0}, {3, 4, 0, 0}};
    Pat *dp;
    CK(hipMalloc(&dp, sizeof(Pat)));
    CK(hipMemcpy(dp, &hp, sizeof(Pat), hipMemcpyHostToDevice));
    Args a{};
    for (int i = 0; i < 5; ++i) a.base[i] = slab + i * stride;
    a.tiles = dt;
    a.pats = dp;
    a.n_items = ntiles * 4;
    CK(hipDeviceSynchronize());
    int cus = 256;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    const size_t lds_cu = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 160 * 1024;

    struct V {
        std::string name;
        int kind;  // 0 bare, 1 meta, 2 persist, 3 pipe, 4 tile
        int cap;   // workgroups (= waves) per CU; 0 = no cap
    };
    std::vector<V> vs;
    const std::vector<int> caps = {0, 8, 10, 12, 16, 24};
    const char *kn[] = {"bare", "meta", "persist", "pipe", "tile"};
    for (int k : {0, 4, 1})
        for (int c : caps) {
            if (k >= 2 && c == 0) continue;
            vs.push_back({std::string(kn[k]) + (c ? " cap " + std::to_string(c) : std::string(" no cap")), k, c});
        }
    auto launch = [&](const V &v) {
        const size_t lds = v.cap ? lds_cu / v.cap - 256 : 0;
        switch (v.kind) {
        case 0: hipLaunchKernelGGL(k_bare, a.n_items, 64, lds, 0, a); break;
        case 1: hipLaunchKernelGGL(k_meta, a.n_items, 64, lds, 0, a); break;
        case 2: hipLaunchKernelGGL(k_persist, cus * v.cap, 64, lds, 0, a); break;
        case 3: hipLaunchKernelGGL(k_pipe, cus * v.cap, 64, lds, 0, a); break;
        case 4: hipLaunchKernelGGL(k_tile, a.n_items, 64, lds, 0, a); break;
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? atoi(argv[1]) : 7, iters = 10;
    std::vector<std::vector<float>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            launch(vs[i]);
            CK(hipGetLastError());
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; ++it) launch(vs[i]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t / iters);
        }
    // correctness of the last launch kind: parity0 = d0^d1^d2
    std::vector<uint8_t> h(4 * 1024 * 1024), d0(h.size()), d1(h.size()), d2(h.size());
    CK(hipMemcpy(h.data(), slab + 3 * stride + L - h.size(), h.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(d0.data(), slab + 0 * stride + L - h.size(), h.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(d1.data(), slab + 1 * stride + L - h.size(), h.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(d2.data(), slab + 2 * stride + L - h.size(), h.size(), hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < h.size(); ++i) bad += h[i] != (uint8_t)(d0[i] ^ d1[i] ^ d2[i]);
    printf("RS(3,2)-shaped 3R:2W, 1 KiB items, 64-lane WGs, %d CUs, tail check %zu bad\n", cus, bad);
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(ms[i].begin(), ms[i].end());
        printf("%-22s median %.4f ms -> %.0f GB/s (best %.0f)\n", vs[i].name.c_str(), ms[i][rounds / 2],
               5.0 * L / (ms[i][rounds / 2] * 1e6), 5.0 * L / (ms[i][0] * 1e6));
    }
    return bad ? 1 : 0;
}
