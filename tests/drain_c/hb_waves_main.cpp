// tests/drain_c/hb_waves_main.cpp -- the host batch's wave planning (cec_hostbatch.inc:
// the pieces, the range-assign / range-max tree and hb_cluster_waves), spliced from the
// shipped source (at the marker in the namespace below) by tests/test_abi.py and run under ASan + UBSan on random
// clusters.  The properties cec_region_multiply_batch relies on:
//   * two overlapping pieces never share a wave;
//   * in a cluster holding a write (add = 0 or a base), a piece of a later job runs in a
//     later wave than every earlier-job piece it overlaps (the sequential chain's order);
//   * an XOR-only cluster uses exactly as many waves as its deepest overlap (greedy
//     colouring of intervals is optimal);
//   * `packed` is false only for a lone write / base piece.
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <random>
#include <vector>

namespace {
// HB_FUNCS
}  // namespace

int main() {
    std::mt19937_64 rng(12345);
    int bad = 0;
    for (int it = 0; it < 4000 && !bad; ++it) {
        const int n = 1 + static_cast<int>(rng() % 60);
        const uintptr_t span = 64 + rng() % 4096;
        const bool writes = rng() % 2;
        std::vector<HbPiece> pc(n);
        for (int i = 0; i < n; ++i) {
            HbPiece &p = pc[i];
            const uintptr_t lo = 0x10000 + rng() % span;
            p.dst = reinterpret_cast<uint8_t *>(lo);
            p.len = 1 + static_cast<uint32_t>(rng() % 300);
            p.kind = writes ? static_cast<uint8_t>(rng() % 3) : kHbXor;
            p.job = i;
            p.wave = -1;
        }
        // the caller hands one cluster's pieces sorted by dst start
        std::vector<int> ids(n);
        for (int i = 0; i < n; ++i) ids[i] = i;
        std::sort(ids.begin(), ids.end(), [&](int a, int b) { return pc[a].dst < pc[b].dst; });
        bool packed = false;
        const int nw = hb_cluster_waves(pc, ids.data(), n, &packed);
        auto meet = [&](const HbPiece &a, const HbPiece &b) {
            const uintptr_t al = reinterpret_cast<uintptr_t>(a.dst), bl = reinterpret_cast<uintptr_t>(b.dst);
            return al < bl + b.len && bl < al + a.len;
        };
        bool any_write = false;
        for (const HbPiece &p : pc) any_write |= p.kind != kHbXor;
        int depth = 0;
        for (int i = 0; i < n; ++i) {
            if (pc[i].wave < 0 || pc[i].wave >= nw) bad = 1;
            int d = 1;
            for (int j = 0; j < n; ++j) {
                if (j == i || !meet(pc[i], pc[j])) continue;
                if (pc[i].wave == pc[j].wave) bad = 2;
                if (any_write && j < i && pc[j].wave >= pc[i].wave) bad = 3;
                // overlap depth at pc[i]'s start
                const uintptr_t x = reinterpret_cast<uintptr_t>(pc[i].dst), jl = reinterpret_cast<uintptr_t>(pc[j].dst);
                if (jl <= x && x < jl + pc[j].len) ++d;
            }
            depth = std::max(depth, d);
        }
        if (!any_write && n > 0 && nw != depth) bad = 4;
        if (packed != !(n == 1 && pc[0].kind != kHbXor)) bad = 5;
        if (bad) printf("iteration %d: property %d (n %d, waves %d, depth %d)\n", it, bad, n, nw, depth);
    }
    if (!bad) printf("ok\n");
    return bad;
}
