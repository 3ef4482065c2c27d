// tests/drain_c/waves_main.cpp -- property check of the drainer's wave colouring on the
// CPU: tests/test_abi.py::test_drain_wave_colouring splices the shipped functions
// (sort_by_addr .. overlap_waves of cocytus_amd/csrc/cec_drain.inc) in at WAVES_FUNCS and
// compiles this under ASan + UBSan.  No two overlapping updates may share a wave; a batch
// of distinct values is one wave; the address sort is ordered.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
typedef struct { const void *buf; uint64_t addr; uint32_t len; uint32_t src_lid; } cec_host_update;
// WAVES_FUNCS

int main() {
    std::mt19937_64 r(5);
    for (int t = 0; t < 3000; ++t) {
        int n = 1 + r() % 200;
        std::vector<cec_host_update> u(n);
        const uint64_t span = 1 + r() % (1ull << (r() % 34));
        for (auto &x : u) { x.addr = r() % span; x.len = r() % 4 ? (uint32_t)(r() % 5000) : 0; x.src_lid = 0; x.buf = nullptr; }
        if (t % 3 == 0) for (int i = 0; i < n; ++i) { u[i].addr = (uint64_t)i * 4098 + (t % 7) * (1ull << 33); u[i].len = 4098; }
        std::vector<int> w;
        int nw = overlap_waves(u.data(), n, w);
        int mx = 0;
        for (int i = 0; i < n; ++i) mx = std::max(mx, w[i]);
        if (mx >= nw) { printf("wave out of range\n"); return 1; }
        for (int i = 0; i < n; ++i) for (int j = i + 1; j < n; ++j) {
            if (!u[i].len || !u[j].len || w[i] != w[j]) continue;
            bool ov = u[i].addr < u[j].addr + u[j].len && u[j].addr < u[i].addr + u[i].len;
            if (ov) { printf("overlap in wave t=%d\n", t); return 1; }
        }
        if (t % 3 == 0 && nw != 1) { printf("fast path missed\n"); return 1; }
    }
    std::vector<cec_host_update> u(70000);
    std::mt19937 g(1); std::vector<int> p(u.size()); for (size_t i=0;i<p.size();++i) p[i]=i; std::shuffle(p.begin(),p.end(),g);
    for (size_t i=0;i<u.size();++i) u[i] = {nullptr, (uint64_t)p[i]*4098, 4098, 0};
    std::vector<cec_host_update> byaddr_check(u);
    std::vector<std::pair<uint64_t,int>> s; sort_by_addr(u.data(), (int)u.size(), s);
    for (size_t i=1;i<s.size();++i) if (s[i-1].first > s[i].first) { printf("not sorted\n"); return 1; }
    printf("ok\n");
}
