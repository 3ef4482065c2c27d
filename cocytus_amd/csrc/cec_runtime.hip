// cec_runtime.hip -- libcocytus_ec.so: the C-ABI of the MI355X erasure-coding path.
//
// Exports (a) the three Jerasure 2.x symbols Cocytus links:
//   galois_w08_region_multiply             (memcached.c:2681,5611,7764,7918; recovery.c:91,123)
//   reed_sol_big_vandermonde_distribution_matrix   (memcached.c:6845)
//   jerasure_invert_matrix                 (memcached.c:7907)
// plus a few same-header helpers, and (b) the batched device API of cocytus_ec.h.
// Every byte of region arithmetic runs in the HIP kernels of cec_kernels.hpp; the
// host side only builds coefficient tables, tile work-lists and launches.  There is
// no CPU fallback: without a gfx950 device the batched API returns CEC_ENODEV and
// the void Jerasure entry point aborts with a message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cocytus_ec.h"
#include "../../include/galois.h"
#include "../../include/jerasure.h"
#include "../../include/reed_sol.h"
#include "cec_kernels.hpp"
#include "gf256.hpp"

#define CEC_API extern "C" __attribute__((visibility("default")))

using namespace cec;

static_assert(sizeof(Tile) == sizeof(cec_extent), "tile layout");
static_assert(CEC_MAX_K <= kPatN, "k capacity");

// ============================================================== errors
static thread_local char g_err[512] = "";

static int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(CEC_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                        __FILE__, __LINE__);                                               \
    } while (0)

[[noreturn]] static void die(const char *what) {
    fprintf(stderr, "libcocytus_ec: fatal: %s\n", what);
    fflush(stderr);
    abort();
}

// ============================================================== device state
struct DevInfo {
    std::once_flag once;
    int status = CEC_ENODEV;
    int cus = 256;
    size_t lds_per_cu = 160 * 1024;  // gfx950
    char msg[256] = "";
};
static DevInfo g_dev[64];
static std::atomic<int> g_engine{CEC_ENGINE_AUTO};

// The engine an op runs with, read once per op (its tables and its kernel must agree):
// the process-wide setting, or under AUTO the LDS engine only where it led PERM by more
// than 2 % on the median of the recorded boxes -- `lds_op`: a decode of values of 64 KiB
// and more -- and PERM for every other op (cocytus_ec.h; DESIGN.md §4 "Engine per op").
// Recorded per thread for cec_last_engine().
static thread_local int t_last_engine = -1;
static int op_engine(bool lds_op) {
    const int e = g_engine.load();
    const int r = e == CEC_ENGINE_AUTO ? (lds_op ? CEC_ENGINE_LDS : CEC_ENGINE_PERM) : e;
    t_last_engine = r;
    return r;
}

static int current_device(int *dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return fail(CEC_ENODEV, "no HIP device visible (libcocytus_ec has no CPU fallback)");
    }
    HIP_TRY(hipGetDevice(dev));
    if (*dev < 0 || *dev >= 64) return fail(CEC_ENODEV, "device ordinal %d out of range", *dev);
    DevInfo &d = g_dev[*dev];
    std::call_once(d.once, [&] {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, *dev) != hipSuccess) {
            snprintf(d.msg, sizeof d.msg, "hipGetDeviceProperties(%d) failed", *dev);
            return;
        }
        if (strncmp(p.gcnArchName, "gfx950", 6) != 0) {
            snprintf(d.msg, sizeof d.msg, "device %d is %s, libcocytus_ec is built for gfx950",
                     *dev, p.gcnArchName);
            return;
        }
        d.cus = p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
        if (p.maxSharedMemoryPerMultiProcessor > 0) d.lds_per_cu = p.maxSharedMemoryPerMultiProcessor;
        d.status = CEC_OK;
    });
    if (d.status != CEC_OK) return fail(d.status, "%s", d.msg);
    return CEC_OK;
}

#include "cec_cache.inc"

static Pattern blank_pattern() {
    Pattern p;
    memset(&p, 0, sizeof p);
    return p;
}

static void set_coef(Pattern &p, int l, int i, int c, int engine) {
    c &= 0xFF;
    p.coef[l][i] = static_cast<uint8_t>(c);
    if (engine != CEC_ENGINE_LDS) {
        const PermTab t = make_perm_tab(c);
        for (int w = 0; w < 5; ++w) p.tab[l][i][w] = t.w[w];
    }
}

// LDS engine: one 256-B product row per distinct coefficient c >= 2 of the pattern,
// row_c[x] = exp[log x + log c] (0 for x = 0), appended to `rows`; the kernel stages
// the pattern's rows into LDS and looks up one byte per byte (cec_kernels.hpp).
static void assign_rows(Pattern &p, std::vector<uint8_t> &rows) {
    int row_of[256];
    for (int &r : row_of) r = -1;
    const size_t base = rows.size() / 256;
    int nr = 0;
    for (int l = 0; l < p.n_out; ++l)
        for (int i = 0; i < p.n_in; ++i) {
            const int c = p.coef[l][i];
            if (c < 2) continue;  // 0 and 1 are uniform branches, no table
            if (row_of[c] < 0) {
                row_of[c] = nr++;
                for (int x = 0; x < 256; ++x)
                    rows.push_back(x ? kGf.exp[kGf.log[x] + kGf.log[c]] : 0);
            }
            p.tab[l][i][0] = static_cast<uint32_t>(row_of[c]) * 256u;
        }
    p.lds_rows = nr;
    p.lds_row_base = static_cast<int32_t>(base);
}

// ============================================================== launch
// `lds`: dynamic LDS bytes of the launch (LDS engine: the largest pattern's rows).
template <int NT, int LT, class Eng, int kAcc, bool kExact, int S = kMaxStreams, bool kSysRel = false>
static void launch_k(const CombineArgsN<S> &a, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((combine_kernel<NT, LT, Eng, kAcc, kExact, S, kSysRel>), dim3(grid),
                       dim3(kBlock >> a.split_shift), lds, s, a);
}

// The 1 x 1 shapes (region multiply-XOR / write, parity apply) with the two-slot
// arguments, for launches whose patterns use slots 0 and 1 only.  narrow_args builds the
// argument block they are passed (the launch-time check reads the same block).
static CombineArgsN<kNarrowStreams> narrow_args(const CombineArgs &w) {
    CombineArgsN<kNarrowStreams> a;
    memset(&a, 0, sizeof a);
    for (int i = 0; i < kNarrowStreams; ++i) a.base[i] = w.base[i];
    a.tiles = w.tiles;
    a.patterns = w.patterns;
    a.rows = w.rows;
    a.implicit_len = w.implicit_len;
    a.n_tiles = w.n_tiles;
    a.split_shift = w.split_shift;
    a.grid = w.grid;
    a.flags = w.flags;
    return a;
}

template <class Eng>
static bool launch_narrow(int acc, const CombineArgsN<kNarrowStreams> &a, int grid, size_t lds, hipStream_t s) {
    const bool rel = (a.flags & kFlagSysRelease) != 0;
    if (acc == kAccAll && rel) launch_k<1, 1, Eng, kAccAll, true, kNarrowStreams, true>(a, grid, lds, s);
    else if (acc == kAccAll) launch_k<1, 1, Eng, kAccAll, true, kNarrowStreams>(a, grid, lds, s);
    else if (acc == kAccNone && rel) launch_k<1, 1, Eng, kAccNone, true, kNarrowStreams, true>(a, grid, lds, s);
    else if (acc == kAccNone) launch_k<1, 1, Eng, kAccNone, true, kNarrowStreams>(a, grid, lds, s);
    else return false;
    return true;
}

// Exact-shape kernels for the hot ops: encode / decode / residual / solve (no RMW,
// up to 8 inputs x 4 outputs), parity apply and region multiply-XOR (1 x 1 RMW),
// diff-update (2 inputs, M parity RMW outputs, optionally + install).
template <class Eng>
static bool launch_exact(int n, int l, int acc, const CombineArgs &a, int grid, size_t lds,
                         hipStream_t s) {
#define CEC_X(N, L, A)                                           \
    if (n == N && l == L && acc == A) {                          \
        launch_k<N, L, Eng, A, true>(a, grid, lds, s);       \
        return true;                                             \
    }
#define CEC_XL(N) CEC_X(N, 1, kAccNone) CEC_X(N, 2, kAccNone) CEC_X(N, 3, kAccNone) CEC_X(N, 4, kAccNone)
    CEC_XL(1) CEC_XL(2) CEC_XL(3) CEC_XL(4) CEC_XL(5) CEC_XL(6) CEC_XL(7) CEC_XL(8)
    CEC_X(1, 1, kAccAll) CEC_X(2, 1, kAccAll) CEC_X(2, 2, kAccAll) CEC_X(2, 3, kAccAll)
    CEC_X(2, 4, kAccAll) CEC_X(2, 2, kAccAllButLast) CEC_X(2, 3, kAccAllButLast)
    CEC_X(2, 4, kAccAllButLast)
#undef CEC_XL
#undef CEC_X
    return false;
}

// The (n_in, n_out, acc) shapes launch_exact instantiates.
static bool has_exact(int n, int l, int acc) {
    if (acc == kAccNone) return n >= 1 && n <= 8 && l >= 1 && l <= 4;
    if (acc == kAccAll) return (n == 1 && l == 1) || (n == 2 && l >= 1 && l <= 4);
    if (acc == kAccAllButLast) return n == 2 && l >= 2 && l <= 4;
    return false;
}

// Capacity kernels for every other shape (guarded, per-pattern counts and modes).
template <class Eng>
static void launch_generic(int nt, int lt, const CombineArgs &a, int grid, size_t lds, hipStream_t s) {
#define CEC_G(NT)                                                                        \
    if (lt <= 1) launch_k<NT, 1, Eng, kAccRuntime, false>(a, grid, lds, s);          \
    else if (lt <= 2) launch_k<NT, 2, Eng, kAccRuntime, false>(a, grid, lds, s);     \
    else launch_k<NT, 4, Eng, kAccRuntime, false>(a, grid, lds, s);
    if (nt <= 2) { CEC_G(2) }
    else if (nt <= 4) { CEC_G(4) }
    else if (nt <= 8) { CEC_G(8) }
    else { CEC_G(16) }
#undef CEC_G
}

// Shape class of the patterns a launch uses (`used`: pattern indices its tiles name;
// NULL = all): exact (n_in, n_out, acc) if they all agree.
static bool exact_shape(const std::vector<Pattern> &pats, const std::vector<char> *used, int *n, int *l,
                        int *acc) {
    const Pattern *p0 = nullptr;
    for (size_t i = 0; i < pats.size(); ++i) {
        if (used && !(*used)[i]) continue;
        const Pattern &p = pats[i];
        if (!p0) {
            p0 = &p;
            continue;
        }
        if (p.n_in != p0->n_in || p.n_out != p0->n_out) return false;
        for (int o = 0; o < p.n_out; ++o)
            if (p.out_mode[o] != p0->out_mode[o]) return false;
    }
    if (!p0) return false;
    int nx = 0;
    for (int o = 0; o < p0->n_out; ++o) nx += p0->out_mode[o] == kModeXor;
    if (nx == 0) *acc = kAccNone;
    else if (nx == p0->n_out) *acc = kAccAll;
    else if (nx == p0->n_out - 1 && p0->out_mode[p0->n_out - 1] == kModeWrite) *acc = kAccAllButLast;
    else return false;
    *n = p0->n_in;
    *l = p0->n_out;
    return true;
}

struct Streams {
    uint8_t *base[kMaxStreams] = {};
};

// One launch over a tile source (plan or implicit region) with a pattern set built for
// `engine` (the patterns' coefficient form and the kernel must agree: the engine is read
// once per op, so a concurrent cec_set_engine cannot split them).
static int run_combine(int dev, const Streams &st, const std::vector<Pattern> &pats,
                       const std::vector<uint8_t> &rows, const cec_plan *plan,
                       uint64_t implicit_len, hipStream_t stream, const std::vector<char> *used, int engine);

// ============================================================== plans
// Tiles of one extent end on 4 KiB boundaries of the arena offset, so interior
// tiles cover whole 128-B lines and only an extent's first / last tile shares a line
// with a neighbouring workgroup (ecalloc packs values at 16-B granularity; tiling
// from each value's start measured 4 % slower on the mixed workload).
static inline size_t tiles_of(uint64_t off, uint32_t len) {
    return len ? static_cast<size_t>((off % kTile + len + kTile - 1) / kTile) : 0;
}
static inline size_t append_tiles(Tile *t, uint64_t off, uint64_t src_off, uint32_t len,
                                  uint32_t pattern) {
    size_t n = 0;
    for (uint32_t o = 0; o < len;) {
        const uint32_t phase = static_cast<uint32_t>((off + o) % kTile);
        const uint32_t step = std::min<uint32_t>(kTile - phase, len - o);
        t[n++] = Tile{off + o, src_off + o, step, pattern};
        o += step;
    }
    return n;
}
// Full tiles whose arena offset sits on a 128-B line (the written side: a line
// written by two workgroups costs more than one read by two).
static inline int64_t count_line_tiles(const Tile *t, size_t n) {
    int64_t c = 0;
    for (size_t i = 0; i < n; ++i) c += t[i].len == kTile && (t[i].off & (kLineBytes - 1)) == 0;
    return c;
}

struct cec_plan {
    int device = -1;
    int n_ext = 0;
    int64_t n_tiles = 0;
    uint64_t total = 0;
    bool overlap = false;
    int64_t n_line_tiles = 0;   // full kTile tiles at a 128-B aligned arena offset
    Tile *d_tiles = nullptr;    // from dev_cache() (owned plans only; views borrow)
    bool owned = false;
    uint32_t max_pattern = 0;       // largest extent pattern (per-op index validation)
    std::vector<Tile> h_tiles;      // kept alive for the async upload
    mutable Tracker uses;           // the streams of the tile upload and of every launch
};

CEC_API int cec_plan_destroy(cec_plan *p) {
    if (!p) return CEC_OK;
    int rc = CEC_OK;
    // only this plan's own work: its upload and its launches on every stream used
    if (hipError_t e = p->uses.wait(p->device); e != hipSuccess)
        rc = fail(CEC_EHIP, "cec_plan_destroy: a launch of this plan failed: %s", hipGetErrorString(e));
    if (p->owned) dev_cache().release(p->device, p->d_tiles, sizeof(Tile) * p->n_tiles);
    delete p;
    return rc;
}

// The caller is destroying `stream`: wait for this plan's work on it and stop tracking it
// (per-connection streams: the tracked list stays bounded by the streams alive).
CEC_API int cec_plan_release_stream(cec_plan *p, void *stream) {
    if (!p) return fail(CEC_EINVAL, "cec_plan_release_stream: plan is NULL");
    if (hipError_t e = p->uses.release(p->device, static_cast<hipStream_t>(stream)); e != hipSuccess)
        return fail(CEC_EHIP, "cec_plan_release_stream: %s", hipGetErrorString(e));
    return CEC_OK;
}
CEC_API int cec_plan_tracked_streams(const cec_plan *p) { return p ? static_cast<int>(p->uses.size()) : 0; }

CEC_API int cec_plan_create(cec_plan **out, const cec_extent *ext, int n, void *stream) {
    if (!out || n < 0 || (n > 0 && !ext)) return fail(CEC_EINVAL, "cec_plan_create: bad args");
    *out = nullptr;
    int dev;
    if (int r = current_device(&dev)) return r;
    cec_plan *p = new (std::nothrow) cec_plan;
    if (!p) return fail(CEC_ENOMEM, "cec_plan_create: host allocation");
    p->device = dev;
    p->n_ext = n;
    for (int e = 0; e < n; ++e) p->max_pattern = std::max(p->max_pattern, ext[e].pattern);
    size_t total_tiles = 0;
    for (int e = 0; e < n; ++e) total_tiles += tiles_of(ext[e].off, ext[e].len);
    p->h_tiles.resize(total_tiles);
    size_t nt = 0;
    for (int e = 0; e < n; ++e) {
        p->total += ext[e].len;
        nt += append_tiles(p->h_tiles.data() + nt, ext[e].off, ext[e].src_off, ext[e].len, ext[e].pattern);
    }
    if (p->h_tiles.size() > 0xFFFFFFFFull) {
        delete p;
        return fail(CEC_EINVAL, "cec_plan_create: more than 2^32 tiles");
    }
    p->n_tiles = static_cast<int64_t>(p->h_tiles.size());
    p->n_line_tiles = count_line_tiles(p->h_tiles.data(), p->h_tiles.size());
    {   // overlap of [off, off+len) among non-empty extents
        std::vector<std::pair<uint64_t, uint64_t>> r;
        r.reserve(n);
        for (int e = 0; e < n; ++e)
            if (ext[e].len) r.emplace_back(ext[e].off, ext[e].off + ext[e].len);
        std::sort(r.begin(), r.end());
        for (size_t i = 1; i < r.size(); ++i)
            if (r[i].first < r[i - 1].second) { p->overlap = true; break; }
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (p->n_tiles > 0) {
        const size_t bytes = sizeof(Tile) * p->n_tiles;
        p->d_tiles = static_cast<Tile *>(dev_cache().acquire(dev, bytes));
        if (!p->d_tiles) {
            delete p;
            return fail(CEC_ENOMEM, "cec_plan_create: %zu bytes of tiles", bytes);
        }
        p->owned = true;
        if (hipMemcpyAsync(p->d_tiles, p->h_tiles.data(), bytes, hipMemcpyHostToDevice, s) != hipSuccess) {
            (void)hipGetLastError();
            cec_plan_destroy(p);
            return fail(CEC_EHIP, "cec_plan_create: tile upload failed");
        }
        p->uses.note(s);  // destroy waits for the upload too
    }
    *out = p;
    return CEC_OK;
}

CEC_API int cec_plan_num_extents(const cec_plan *p) { return p ? p->n_ext : 0; }
CEC_API int64_t cec_plan_num_tiles(const cec_plan *p) { return p ? p->n_tiles : 0; }
CEC_API uint64_t cec_plan_total_bytes(const cec_plan *p) { return p ? p->total : 0; }

// Workgroups per tile (log2).  Full tiles on 128-B lines stream fastest as four
// 64-lane workgroups (finer dispatch, every wave equal work).  A plan that is mostly
// small or line-misaligned tiles keeps one 256-lane workgroup per tile: splitting
// those multiplies empty workgroups and partial lines written by two workgroups
// (measured: DESIGN.md section 4).  CEC_SPLIT_SHIFT=0..2 pins the choice.
static uint32_t split_shift_for(const Streams &st, const cec_plan *plan) {
    static const int forced = [] {
        const char *e = getenv("CEC_SPLIT_SHIFT");
        return e && *e ? std::min(2, std::max(0, atoi(e))) : -1;
    }();
    if (forced >= 0) return static_cast<uint32_t>(forced);
    uintptr_t mis = 0;
    for (int i = 0; i < kMaxStreams; ++i) mis |= reinterpret_cast<uintptr_t>(st.base[i]);
    const bool full = plan ? plan->n_line_tiles * 4 >= plan->n_tiles * 3 : true;
    return full && (mis & (kLineBytes - 1)) == 0 ? 2u : 0u;
}

// Waves per CU a launch may hold (0 = as many as fit).  Fewer streaming waves per CU
// keep fewer HBM requests in flight; the cap is applied by sizing each workgroup's
// dynamic LDS so that only cap / (waves per workgroup) workgroups fit on a CU.
// CEC_WAVES_PER_CU overrides it (measurement).
static std::atomic<int> g_waves_per_cu{[] {
    const char *e = getenv("CEC_WAVES_PER_CU");
    return e && *e ? std::max(0, atoi(e)) : 0;
}()};
static int waves_per_cu_cap() { return g_waves_per_cu.load(std::memory_order_relaxed); }

static size_t occupancy_lds(int dev, uint32_t split_shift) {
    const int cap = waves_per_cu_cap();
    if (cap <= 0) return 0;
    const int waves_per_wg = (kBlock >> split_shift) / 64;
    const int wgs = std::max(1, cap / std::max(1, waves_per_wg));
    const size_t per_cu = g_dev[dev].lds_per_cu;
    const size_t lds = per_cu / static_cast<size_t>(wgs);
    return std::min<size_t>(65536, lds > 256 ? lds - 256 : 0);  // strictly below the boundary
}

// Store policy of a launch (kFlagWriteThrough).  Write-through (sc1) stores finish the
// launches of up to 512 MiB of streamed bytes sooner, non-temporal stores the larger
// ones.  RS(3,2) 4 KiB step, bench.py's strong-scaling shares, 3 processes per policy on
// one box (profiles/r03_evidence/store_policy_ab/): encode / decode us
//   8,192 stripes   nt 29.9-31.7 / 23.6-23.9   wt 27.5-28.6 / 22.3-22.6
//  16,384 stripes   nt 54.0-55.3 / 45.5-45.6   wt 53.4-54.0 / 41.0-41.6
//  32,768 stripes   nt 105.9-106.2 / 88.1-88.6 wt 112.5-112.7 / 81.1-81.8
//  65,536 stripes   nt 208.0-212.2 / 178.0-178.3  wt 223.3-224.8 / 184.8-186.1
// i.e. write-through wins at <= 335 MB (encode) and <= 537 MB (decode) per launch and
// loses at 671 MB (encode) and above.  Auto: write-through when the launch streams at
// most g_wt_max_bytes (reads + writes).  CEC_STORE_POLICY=nt|wt|auto and
// CEC_WT_MAX_BYTES override (measurement).
enum { kStoreAuto = 0, kStoreNt = 1, kStoreWt = 2 };
// An unknown value (e.g. "WT") is reported on stderr once and ignored (auto).
static const int g_store_policy = [] {
    const char *e = getenv("CEC_STORE_POLICY");
    if (!e || !*e || !strcmp(e, "auto")) return static_cast<int>(kStoreAuto);
    if (!strcmp(e, "wt")) return static_cast<int>(kStoreWt);
    if (!strcmp(e, "nt")) return static_cast<int>(kStoreNt);
    fprintf(stderr, "libcocytus_ec: CEC_STORE_POLICY=%s is not nt, wt or auto; using auto\n", e);
    return static_cast<int>(kStoreAuto);
}();
static const uint64_t g_wt_max_bytes = [] {
    const uint64_t dflt = uint64_t(512) << 20;
    const char *e = getenv("CEC_WT_MAX_BYTES");
    if (!e || !*e) return dflt;
    // strtoull alone would take "-1" as 2^64 - 1 and skip leading blanks: a byte count is
    // digits only (decimal, 0x hex or 0 octal), in range
    char *end = nullptr;
    errno = 0;
    const unsigned long long v = (*e >= '0' && *e <= '9') ? strtoull(e, &end, 0) : 0;
    if (!(*e >= '0' && *e <= '9') || !end || *end || errno == ERANGE) {
        fprintf(stderr, "libcocytus_ec: CEC_WT_MAX_BYTES=%s is not a byte count; using %llu\n", e,
                static_cast<unsigned long long>(dflt));
        return dflt;
    }
    return static_cast<uint64_t>(v);
}();
// The store policy in force (tests: every kernel kind runs under each).
CEC_API int cec_internal_store_policy(uint64_t *wt_max_bytes) {
    if (wt_max_bytes) *wt_max_bytes = g_wt_max_bytes;
    return g_store_policy;
}
static bool write_through(uint64_t n_tiles, int streams) {
    if (g_store_policy != kStoreAuto) return g_store_policy == kStoreWt;
    return n_tiles * kTile * static_cast<uint64_t>(streams) <= g_wt_max_bytes;
}

// The kernel a pattern set takes: capacities, LDS rows, and the exact shape if every
// pattern the launch uses has the same one.
struct LaunchShape {
    int nt = 1, lt = 0, max_rows = 0;
    bool exact = false;
    int en = 0, el = 0, eacc = 0;
    int streams = 0;  // 1 + the highest stream slot a used pattern names
};

static LaunchShape launch_shape(const std::vector<Pattern> &pats, const std::vector<char> *used) {
    LaunchShape sh;
    for (size_t i = 0; i < pats.size(); ++i) {
        if (used && !(*used)[i]) continue;
        sh.nt = std::max(sh.nt, pats[i].n_in);
        sh.lt = std::max(sh.lt, pats[i].n_out);
        sh.max_rows = std::max(sh.max_rows, pats[i].lds_rows);
        for (int j = 0; j < pats[i].n_in; ++j) sh.streams = std::max(sh.streams, pats[i].in_stream[j] + 1);
        for (int j = 0; j < pats[i].n_out; ++j) sh.streams = std::max(sh.streams, pats[i].out_stream[j] + 1);
    }
    sh.exact = exact_shape(pats, used, &sh.en, &sh.el, &sh.eacc);
    return sh;
}

// One launch over n_tiles (> 0) tiles of a plan or an implicit region, with the tables
// (n_pats patterns, then the LDS engine's rows) already on the device.  The caller
// checks hipGetLastError.
// *released: whether every wave of the launch ends with a system-scope release
// (kFlagSysRelease asked for, and honoured: only the narrow 1 x 1 launches carry it).
// hpats / used: the host copies of the launch's patterns and which of them its tiles
// name (NULL: all), for the stream check below.
enum KernelKind { kKindNarrow, kKindExact, kKindGeneric };

// Launch-time check of the argument block a kernel of `kind` is passed: every stream
// slot a used pattern names must be one the block carries (below 2 for the narrow
// kernels, whose block is narrow_args' copy of the first two slots; below kMaxStreams
// otherwise) and hold a non-NULL base there.  Which arena the op meant for each slot is
// decided by the op itself (it fills the slots); this check catches a kernel choice or
// an argument block that cannot serve the patterns -- a slot the kernel's block does not
// have, or an empty one -- which would otherwise fault the GPU.  A failure is refused.
static bool stream_layout_ok(const uint8_t *const *bases, int slots, const Pattern *hpats, size_t n_pats,
                             const std::vector<char> *used) {
    for (size_t q = 0; q < n_pats; ++q) {
        if (used && (q >= used->size() || !(*used)[q])) continue;
        const Pattern &p = hpats[q];
        for (int i = 0; i < p.n_in; ++i)
            if (p.in_stream[i] >= slots || !bases[p.in_stream[i]]) return false;
        for (int l = 0; l < p.n_out; ++l)
            if (p.out_stream[l] >= slots || !bases[p.out_stream[l]]) return false;
    }
    return true;
}

static bool layout_ok_for(KernelKind kind, const CombineArgs &a, const Pattern *hpats, size_t n_pats,
                          const std::vector<char> *used) {
    if (kind == kKindNarrow) {
        const CombineArgsN<kNarrowStreams> na = narrow_args(a);
        return stream_layout_ok(na.base, kNarrowStreams, hpats, n_pats, used);
    }
    return stream_layout_ok(a.base, kMaxStreams, hpats, n_pats, used);
}

static int launch_combine(int dev, const Streams &st, const uint8_t *tables, size_t n_pats,
                          const LaunchShape &sh, bool lds, const cec_plan *plan, uint64_t implicit_len,
                          uint64_t n_tiles, hipStream_t stream, const Pattern *hpats,
                          const std::vector<char> *used, uint32_t flags = 0, bool *released = nullptr) {
    CombineArgs a;
    memset(&a, 0, sizeof a);
    a.flags = flags | (write_through(n_tiles, sh.nt + sh.lt) ? kFlagWriteThrough : 0u);
    // Which kernel runs: the exact-shape one if the shape has an instantiation, the narrow
    // two-slot one for 1 x 1 launches over slots 0 and 1, else a capacity kernel.
    const bool exact_k = sh.exact && has_exact(sh.en, sh.el, sh.eacc);
    const KernelKind kind =
        exact_k && sh.en == 1 && sh.el == 1 && sh.streams <= kNarrowStreams &&
                (sh.eacc == kAccAll || sh.eacc == kAccNone)
            ? kKindNarrow
            : exact_k ? kKindExact : kKindGeneric;
    for (int i = 0; i < kMaxStreams; ++i) a.base[i] = st.base[i];
    if (!layout_ok_for(kind, a, hpats, n_pats, used))
        return fail(CEC_EINVAL, "internal: a launch's argument block cannot serve its patterns "
                                "(kind %d, %d x %d); not launched", static_cast<int>(kind), sh.en, sh.el);
    if (plan) a.tiles = plan->d_tiles;
    else a.implicit_len = implicit_len;
    a.patterns = reinterpret_cast<const Pattern *>(tables);
    a.rows = tables + n_pats * sizeof(Pattern);
    a.n_tiles = static_cast<uint32_t>(n_tiles);
    // One workgroup per (part of a) tile, dispatched in tile order, so the set of
    // tiles in flight is a contiguous window of the arenas (measured 5-12 % over a
    // persistent grid-stride grid: DESIGN.md).  The LDS engine stages its pattern's
    // product rows per workgroup (512 B for an RS(3,2) encode, from L2).
    a.split_shift = split_shift_for(st, plan);
    const size_t lds_bytes = std::max(lds ? static_cast<size_t>(sh.max_rows) * 256 : 0,
                                      occupancy_lds(dev, a.split_shift));
    // A dispatch holds at most 2^32 - 1 work items per dimension: past that (more than
    // 64 GiB of tiles per stream) workgroups walk the rest grid-stride.
    const uint64_t max_wgs = 0xFFFFFFFFull / (kBlock >> a.split_shift);
    const int grid = static_cast<int>(std::min<uint64_t>(n_tiles << a.split_shift, max_wgs));
    a.grid = static_cast<uint32_t>(grid);
    bool ok;
    if (kind == kKindNarrow) {
        const CombineArgsN<kNarrowStreams> na = narrow_args(a);
        ok = lds ? launch_narrow<LdsEngine>(sh.eacc, na, grid, lds_bytes, stream)
                 : launch_narrow<PermEngine>(sh.eacc, na, grid, lds_bytes, stream);
    } else if (kind == kKindExact) {
        ok = lds ? launch_exact<LdsEngine>(sh.en, sh.el, sh.eacc, a, grid, lds_bytes, stream)
                 : launch_exact<PermEngine>(sh.en, sh.el, sh.eacc, a, grid, lds_bytes, stream);
    } else {
        if (lds) launch_generic<LdsEngine>(sh.nt, sh.lt, a, grid, lds_bytes, stream);
        else launch_generic<PermEngine>(sh.nt, sh.lt, a, grid, lds_bytes, stream);
        ok = true;
    }
    if (!ok) return fail(CEC_EINVAL, "internal: no %s kernel for %d x %d", kind == kKindNarrow ? "narrow" : "exact",
                         sh.en, sh.el);
    if (released) *released = kind == kKindNarrow && (flags & kFlagSysRelease) != 0;
    return CEC_OK;
}

// Test hook (cec_internal_fail_launch): the calling thread's next `after` launches run, the
// one after them is refused as a HIP failure, then the hook disarms.  -1: off.
static thread_local int t_fail_after = -1;
CEC_API int cec_internal_fail_launch(int after) {
    t_fail_after = after < 0 ? -1 : after;
    return CEC_OK;
}

static int run_combine(int dev, const Streams &st, const std::vector<Pattern> &pats,
                       const std::vector<uint8_t> &rows, const cec_plan *plan,
                       uint64_t implicit_len, hipStream_t stream, const std::vector<char> *used, int engine) {
    if (t_fail_after == 0) {
        t_fail_after = -1;
        return fail(CEC_EHIP, "injected launch failure (cec_internal_fail_launch)");
    }
    if (t_fail_after > 0) --t_fail_after;
    uint64_t n_tiles;
    if (plan) {
        if (plan->device != dev)
            return fail(CEC_EINVAL, "plan built on device %d used on device %d", plan->device, dev);
        n_tiles = static_cast<uint64_t>(plan->n_tiles);
    } else {
        n_tiles = (implicit_len + kTile - 1) / kTile;
        if (n_tiles > 0xFFFFFFFFull) return fail(CEC_EINVAL, "region too large");
    }
    if (n_tiles == 0 || pats.empty()) return CEC_OK;
    const LaunchShape sh = launch_shape(pats, used);
    if (sh.lt == 0) return CEC_OK;
    // Patterns and the LDS engine's product rows are uploaded as one blob: rows follow
    // the patterns (16-B aligned: sizeof(Pattern) is a multiple of 16).
    std::string key(reinterpret_cast<const char *>(pats.data()), pats.size() * sizeof(Pattern));
    key.append(reinterpret_cast<const char *>(rows.data()), rows.size());
    PatEntry *entry = nullptr;
    if (int r = pattern_get(dev, std::move(key), stream, &entry)) return r;
    const int rc = launch_combine(dev, st, entry->d, pats.size(), sh, engine == CEC_ENGINE_LDS, plan,
                                  implicit_len, n_tiles, stream, pats.data(), used);
    // the plan's streams, for its destroy (host-side only); the tables may be evicted
    // again once the launch is enqueued (eviction synchronises the device)
    if (plan) plan->uses.note(stream);
    pattern_done(entry);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return CEC_OK;
}

// Logical pattern with arbitrarily many outputs, before splitting.
struct Combo {
    int n_in = 0;
    uint8_t in_stream[kPatN] = {};
    uint8_t in_src[kPatN] = {};
    struct Out {
        uint8_t stream, src, mode;
        int coef[kPatN];
    };
    std::vector<Out> outs;  // install output (if any) is last
};

// The patterns of launch g of a combo list: outputs [4g, 4g+4) of every combo (an
// install output is last in `outs`, so it runs in the final launch after every group
// read old bytes), with the engine's coefficient form (and LDS rows).
static void build_patterns(const std::vector<Combo> &combos, size_t g, int engine, std::vector<Pattern> &pats,
                           std::vector<uint8_t> &rows) {
    pats.reserve(combos.size());
    for (const Combo &c : combos) {
        Pattern p = blank_pattern();
        p.n_in = c.n_in;
        for (int i = 0; i < c.n_in; ++i) {
            p.in_stream[i] = c.in_stream[i];
            p.in_src[i] = c.in_src[i];
        }
        const size_t n = c.outs.size();
        const size_t lo = g * kPatL, hi = std::min(n, lo + kPatL);
        int no = 0;
        for (size_t o = lo; o < hi; ++o, ++no) {
            const Combo::Out &q = c.outs[o];
            p.out_stream[no] = q.stream;
            p.out_src[no] = q.src;
            p.out_mode[no] = q.mode;
            for (int i = 0; i < c.n_in; ++i) set_coef(p, no, i, q.coef[i], engine);
        }
        p.n_out = no;
        if (engine == CEC_ENGINE_LDS) assign_rows(p, rows);
        pats.push_back(p);
    }
}

// `used`: which combos the launch's tiles name (NULL = all; a persistent pattern table
// may hold more than one launch uses: the kernel shape is chosen from the used ones).
// `lds_op`: the op AUTO runs with the LDS engine (op_engine).
static int run_combos(int dev, const Streams &st, const std::vector<Combo> &combos,
                      const cec_plan *plan, uint64_t implicit_len, hipStream_t stream,
                      const std::vector<char> *used = nullptr, bool lds_op = false) {
    size_t max_out = 0;
    for (const Combo &c : combos) max_out = std::max(max_out, c.outs.size());
    const int engine = op_engine(lds_op);
    const size_t groups = (max_out + kPatL - 1) / kPatL;
    for (size_t g = 0; g < groups; ++g) {
        std::vector<Pattern> pats;
        std::vector<uint8_t> rows;
        build_patterns(combos, g, engine, pats, rows);
        if (int r = run_combine(dev, st, pats, rows, plan, implicit_len, stream, used, engine)) return r;
    }
    return CEC_OK;
}

static int check_code(int k, int m, const int *matrix) {
    if (k < 1 || k > CEC_MAX_K || m < 1 || m > CEC_MAX_M || k + m > 32)
        return fail(CEC_EINVAL, "unsupported code k=%d m=%d (1<=k<=%d, 1<=m<=%d, k+m<=32)", k, m,
                    CEC_MAX_K, CEC_MAX_M);
    if (!matrix) return fail(CEC_EINVAL, "matrix is NULL");
    for (int i = 0; i < (k + m) * k; ++i)
        if (matrix[i] < 0 || matrix[i] > 255)
            return fail(CEC_EINVAL, "matrix entry %d = %d outside GF(2^8)", i, matrix[i]);
    return CEC_OK;
}

#define MATRIX(x, y) matrix[(x) * k + (y)]

// ============================================================== arena layout
CEC_API size_t cec_arena_stride(size_t bytes) {
    size_t pages = (bytes + kTile - 1) / kTile;
    if (pages % 2 == 0) ++pages;  // odd number of 4 KiB pages between arena bases
    return pages * kTile;
}

CEC_API int cec_arenas_alloc(int count, size_t bytes, uint8_t **arenas, void **slab) {
    if (count < 1 || !arenas || !slab) return fail(CEC_EINVAL, "cec_arenas_alloc: bad args");
    *slab = nullptr;
    int dev;
    if (int r = current_device(&dev)) return r;
    const size_t stride = cec_arena_stride(bytes);
    uint8_t *base = nullptr;
    if (hipMalloc(&base, stride * static_cast<size_t>(count)) != hipSuccess) {
        (void)hipGetLastError();
        return fail(CEC_ENOMEM, "cec_arenas_alloc: %d x %zu bytes", count, stride);
    }
    for (int i = 0; i < count; ++i) arenas[i] = base + static_cast<size_t>(i) * stride;
    *slab = base;
    return CEC_OK;
}

CEC_API int cec_arenas_free(void *slab) {
    if (slab) HIP_TRY(hipFree(slab));
    return CEC_OK;
}

// ============================================================== runtime API
CEC_API const char *cec_version(void) { return "cocytus_ec 0.1 (gfx950)"; }
CEC_API const char *cec_last_error(void) { return g_err; }
CEC_API int cec_device_check(void) {
    int dev;
    return current_device(&dev);
}
CEC_API int cec_set_engine(cec_engine e) {
    if (e != CEC_ENGINE_PERM && e != CEC_ENGINE_LDS && e != CEC_ENGINE_AUTO)
        return fail(CEC_EINVAL, "bad engine %d", e);
    g_engine.store(e);
    return CEC_OK;
}
CEC_API cec_engine cec_get_engine(void) { return static_cast<cec_engine>(g_engine.load()); }
CEC_API int cec_last_engine(void) { return t_last_engine; }

// Test hook: the launch-time check (layout_ok_for) on one pattern, as launch_combine
// runs it, for a narrow or a full argument block built from `bases`.  Host only.
CEC_API int cec_internal_check_launch_layout(int narrow, const int *in_slots, int n_in, const int *out_slots,
                                             int n_out, const void *const *bases, int n_bases) {
    if (n_in < 0 || n_in > kPatN || n_out < 0 || n_out > kPatL || n_bases < 0 || n_bases > kMaxStreams ||
        (n_in && !in_slots) || (n_out && !out_slots) || (n_bases && !bases))
        return fail(CEC_EINVAL, "cec_internal_check_launch_layout: bad args");
    Pattern p = blank_pattern();
    p.n_in = n_in;
    p.n_out = n_out;
    for (int i = 0; i < n_in; ++i) {
        if (in_slots[i] < 0 || in_slots[i] >= kMaxStreams) return fail(CEC_EINVAL, "slot %d", in_slots[i]);
        p.in_stream[i] = static_cast<uint8_t>(in_slots[i]);
    }
    for (int l = 0; l < n_out; ++l) {
        if (out_slots[l] < 0 || out_slots[l] >= kMaxStreams) return fail(CEC_EINVAL, "slot %d", out_slots[l]);
        p.out_stream[l] = static_cast<uint8_t>(out_slots[l]);
    }
    CombineArgs a;
    memset(&a, 0, sizeof a);
    for (int i = 0; i < n_bases; ++i) a.base[i] = static_cast<uint8_t *>(const_cast<void *>(bases[i]));
    if (!layout_ok_for(narrow ? kKindNarrow : kKindExact, a, &p, 1, nullptr))
        return fail(CEC_EINVAL, "internal: a launch's argument block cannot serve its patterns; not launched");
    return CEC_OK;
}
CEC_API int cec_set_waves_per_cu(int waves_per_cu) {
    if (waves_per_cu < 0 || waves_per_cu > 64) return fail(CEC_EINVAL, "bad waves_per_cu %d", waves_per_cu);
    g_waves_per_cu.store(waves_per_cu);
    return CEC_OK;
}
CEC_API int cec_get_waves_per_cu(void) { return waves_per_cu_cap(); }

// ============================================================== ops
// Region multiply (one input, one output, an implicit region) without the generic path:
// the tables of a thread's last (device, multby, add, engine) stay pinned in the cache
// and memoised, so a call skips building, copying and hashing its 1.7 KiB pattern and
// the lookup (tools/dropin_breakdown.hip: 3.4 us of host time per call against 0.9 us
// for an empty launch).  The memo is used only once the tables' upload is known
// complete (until then the cache orders each launch after it), and never while
// capturing (the cache then marks the tables).
namespace {
struct RegionMemo {
    int dev = -1, key = -1;
    PatEntry *e = nullptr;  // pinned while memoised
    LaunchShape shape;
    Pattern pat;            // the host copy (launch_combine's stream check)
    ~RegionMemo() {
        if (e) pattern_done(e);
    }
};
thread_local RegionMemo t_region;
}  // namespace

// `plain`: s is known not to be capturing (the drop-in's private stream).
// flags / *released: see launch_combine (the 1 x 1 region launches honour the release).
static int region_launch(int dev, const void *src, int multby, size_t n, void *dst, int add, hipStream_t s,
                         bool plain, uint32_t flags = 0, bool *released = nullptr) {
    const uint64_t n_tiles = (n + kTile - 1) / kTile;
    if (n_tiles > 0xFFFFFFFFull) return fail(CEC_EINVAL, "region too large");
    const int engine = op_engine(false);
    const int key = (engine << 9) | (add ? 256 : 0) | multby;
    const bool capturing = !plain && stream_capturing(s);
    RegionMemo &m = t_region;
    Streams st;
    st.base[0] = static_cast<uint8_t *>(const_cast<void *>(src));
    st.base[1] = static_cast<uint8_t *>(dst);
    if (!(m.e && m.dev == dev && m.key == key && !capturing && m.e->up_done.load(std::memory_order_acquire))) {
        Combo cb;
        cb.n_in = 1;
        cb.in_stream[0] = 0;
        Combo::Out o{};
        o.stream = 1;
        o.mode = add ? kModeXor : kModeWrite;
        o.coef[0] = multby;
        cb.outs.push_back(o);
        std::vector<Pattern> pats;
        std::vector<uint8_t> rows;
        build_patterns({cb}, 0, engine, pats, rows);
        std::string k(reinterpret_cast<const char *>(pats.data()), pats.size() * sizeof(Pattern));
        k.append(reinterpret_cast<const char *>(rows.data()), rows.size());
        PatEntry *e = nullptr;
        if (int r = pattern_get(dev, std::move(k), s, &e)) return r;
        if (capturing) {  // tables now marked captured: pinned for this launch only
            const int rc = launch_combine(dev, st, e->d, 1, launch_shape(pats, nullptr), engine == CEC_ENGINE_LDS,
                                          nullptr, n, n_tiles, s, pats.data(), nullptr, flags, released);
            pattern_done(e);
            if (rc) return rc;
            HIP_TRY(hipGetLastError());
            return CEC_OK;
        }
        if (m.e) pattern_done(m.e);  // this launch's pin becomes the memo's
        m.dev = dev;
        m.key = key;
        m.e = e;
        m.shape = launch_shape(pats, nullptr);
        m.pat = pats[0];
    }
    if (int rc = launch_combine(dev, st, m.e->d, 1, m.shape, engine == CEC_ENGINE_LDS, nullptr, n, n_tiles, s,
                                &m.pat, nullptr, flags, released))
        return rc;
    HIP_TRY(hipGetLastError());
    return CEC_OK;
}

CEC_API int cec_region_multiply(const void *src, int multby, size_t nbytes, void *dst, int add,
                                void *stream) {
    if (!src || multby < 0 || multby > 255) return fail(CEC_EINVAL, "cec_region_multiply: bad args");
    int dev;
    if (int r = current_device(&dev)) return r;
    if (nbytes == 0) return CEC_OK;
    if (!dst) {
        dst = const_cast<void *>(src);
        add = 0;
    }
    if (add && multby == 0) return CEC_OK;
    return region_launch(dev, src, multby, nbytes, dst, add, static_cast<hipStream_t>(stream), false);
}

// AUTO's value-size rule for the decode: values of 64 KiB and more run the LDS engine,
// smaller ones (with erasures varying per value) PERM.  Measured on two boxes, two rounds
// each (profiles/r03_evidence/engine_auto/workloads_box*/; a third box agreed): at 64 KiB,
// 1 MiB and the mixed 256 B - 1 MiB batch the LDS engine led the rotating decode by
// 2.5-3.7 %, at 4 KiB PERM led it by 2-3 %.  The encode is within +-2 % at every size
// (LDS ahead by 0-1.6 % on large values, a tie at 4 KiB), so it runs PERM throughout.
static bool large_values(const cec_plan *plan) {
    return !plan || plan->total >= (uint64_t(64) << 10) * static_cast<uint64_t>(std::max(plan->n_ext, 1));
}

static int encode_common(int k, int m, const int *matrix, const uint8_t *const *data,
                         uint8_t *const *parity, const cec_plan *plan, uint64_t len,
                         void *stream) {
    if (int r = check_code(k, m, matrix)) return r;
    if (!data || !parity) return fail(CEC_EINVAL, "cec_encode: NULL arena array");
    int dev;
    if (int r = current_device(&dev)) return r;
    Streams st;
    Combo c;
    c.n_in = k;
    for (int j = 0; j < k; ++j) {
        if (!data[j]) return fail(CEC_EINVAL, "cec_encode: data[%d] is NULL", j);
        st.base[j] = const_cast<uint8_t *>(data[j]);
        c.in_stream[j] = static_cast<uint8_t>(j);
    }
    for (int p = 0; p < m; ++p) {
        if (!parity[p]) continue;  // a lost parity is simply not produced
        st.base[k + p] = parity[p];
        Combo::Out o{};
        o.stream = static_cast<uint8_t>(k + p);
        o.mode = kModeWrite;
        for (int j = 0; j < k; ++j) o.coef[j] = MATRIX(k + p, j);
        c.outs.push_back(o);
    }
    return run_combos(dev, st, {c}, plan, len, static_cast<hipStream_t>(stream));
}

// Ops with one pattern index every tile's pattern field into a one-entry table: it must be 0.
static int single_pattern_plan(const cec_plan *plan, const char *op) {
    if (plan->n_ext && plan->max_pattern != 0)
        return fail(CEC_EINVAL, "%s: extent pattern %u, must be 0 for this op", op, plan->max_pattern);
    return CEC_OK;
}

CEC_API int cec_encode(int k, int m, const int *matrix, const uint8_t *const *data,
                       uint8_t *const *parity, const cec_plan *plan, void *stream) {
    if (!plan) return fail(CEC_EINVAL, "cec_encode: plan is NULL");
    if (int r = single_pattern_plan(plan, "cec_encode")) return r;
    return encode_common(k, m, matrix, data, parity, plan, 0, stream);
}

CEC_API int cec_encode_region(int k, int m, const int *matrix, const uint8_t *const *data,
                              uint8_t *const *parity, size_t len, void *stream) {
    return encode_common(k, m, matrix, data, parity, nullptr, len, stream);
}

CEC_API int cec_diff_update(int k, int m, const int *matrix, uint8_t *const *data,
                            const uint8_t *staging, uint8_t *const *parity, int install,
                            const cec_plan *plan, void *stream) {
    if (int r = check_code(k, m, matrix)) return r;
    if (!plan || !data || !staging || !parity) return fail(CEC_EINVAL, "cec_diff_update: NULL arg");
    if (plan->overlap) return fail(CEC_EOVERLAP, "cec_diff_update: plan extents overlap");
    if (plan->n_ext && plan->max_pattern >= static_cast<uint32_t>(k))
        return fail(CEC_EINVAL, "cec_diff_update: an extent names source shard %u (k = %d)", plan->max_pattern, k);
    int dev;
    if (int r = current_device(&dev)) return r;
    Streams st;
    for (int j = 0; j < k; ++j) {
        if (!data[j]) return fail(CEC_EINVAL, "cec_diff_update: data[%d] is NULL", j);
        st.base[j] = data[j];
    }
    for (int p = 0; p < m; ++p) st.base[k + p] = parity[p];
    st.base[k + m] = const_cast<uint8_t *>(staging);
    std::vector<Combo> combos(k);
    for (int j = 0; j < k; ++j) {
        Combo &c = combos[j];
        c.n_in = 2;
        c.in_stream[0] = static_cast<uint8_t>(j);      // old bytes, arena offset
        c.in_stream[1] = static_cast<uint8_t>(k + m);  // new value, staging offset
        c.in_src[1] = 1;
        for (int p = 0; p < m; ++p) {
            if (!parity[p]) continue;  // lost parity: skipped like memcached.c:2692-2694
            Combo::Out o{};
            o.stream = static_cast<uint8_t>(k + p);
            o.mode = kModeXor;
            o.coef[0] = o.coef[1] = MATRIX(k + p, j);
            c.outs.push_back(o);
        }
        if (install) {
            Combo::Out o{};
            o.stream = static_cast<uint8_t>(j);
            o.mode = kModeWrite;
            o.coef[0] = 0;
            o.coef[1] = 1;
            c.outs.push_back(o);
        }
    }
    // AUTO: PERM.  The LDS engine's diff-update was within +-3 % of PERM either way over
    // the recorded boxes (median margin under 1 %; DESIGN.md §4 "Engine per op").
    return run_combos(dev, st, combos, plan, 0, static_cast<hipStream_t>(stream));
}

CEC_API int cec_set_diff(int k, const uint8_t *const *data, const uint8_t *staging, uint8_t *diff,
                         const cec_plan *plan, void *stream) {
    if (k < 1 || k > CEC_MAX_K || !plan || !data || !staging || !diff)
        return fail(CEC_EINVAL, "cec_set_diff: bad args");
    if (plan->n_ext && plan->max_pattern >= static_cast<uint32_t>(k))
        return fail(CEC_EINVAL, "cec_set_diff: an extent names source shard %u (k = %d)", plan->max_pattern, k);
    int dev;
    if (int r = current_device(&dev)) return r;
    Streams st;
    for (int j = 0; j < k; ++j) {
        if (!data[j]) return fail(CEC_EINVAL, "cec_set_diff: data[%d] is NULL", j);
        st.base[j] = const_cast<uint8_t *>(data[j]);
    }
    st.base[k] = const_cast<uint8_t *>(staging);
    st.base[k + 1] = diff;
    std::vector<Combo> combos(k);
    for (int j = 0; j < k; ++j) {
        Combo &c = combos[j];
        c.n_in = 2;
        c.in_stream[0] = static_cast<uint8_t>(j);
        c.in_stream[1] = static_cast<uint8_t>(k);
        c.in_src[1] = 1;
        Combo::Out o{};
        o.stream = static_cast<uint8_t>(k + 1);
        o.src = 1;
        o.mode = kModeWrite;
        o.coef[0] = o.coef[1] = 1;
        c.outs.push_back(o);
    }
    return run_combos(dev, st, combos, plan, 0, static_cast<hipStream_t>(stream));
}

CEC_API int cec_apply_diffs(int k, int m, const int *matrix, int lid_self, const uint8_t *diffs,
                            uint8_t *parity, const cec_plan *plan, void *stream) {
    if (int r = check_code(k, m, matrix)) return r;
    if (lid_self < k || lid_self >= k + m || !diffs || !parity || !plan)
        return fail(CEC_EINVAL, "cec_apply_diffs: bad args (lid_self=%d)", lid_self);
    if (plan->overlap) return fail(CEC_EOVERLAP, "cec_apply_diffs: plan extents overlap");
    if (plan->n_ext && plan->max_pattern >= static_cast<uint32_t>(k))
        return fail(CEC_EINVAL, "cec_apply_diffs: an extent names source shard %u (k = %d)", plan->max_pattern, k);
    int dev;
    if (int r = current_device(&dev)) return r;
    Streams st;
    st.base[0] = const_cast<uint8_t *>(diffs);
    st.base[1] = parity;
    std::vector<Combo> combos(k);
    for (int j = 0; j < k; ++j) {
        Combo &c = combos[j];
        c.n_in = 1;
        c.in_stream[0] = 0;
        c.in_src[0] = 1;
        Combo::Out o{};
        o.stream = 1;
        o.mode = kModeXor;
        o.coef[0] = MATRIX(lid_self, j);
        c.outs.push_back(o);
    }
    return run_combos(dev, st, combos, plan, 0, static_cast<hipStream_t>(stream));
}

static int mask_ok(int k, int m, uint32_t mask) {
    if (k + m < 32 && (mask >> (k + m)) != 0) return 0;
    return __builtin_popcount(mask) == k;
}

CEC_API int cec_residual(int k, int m, const int *matrix, int lid_self, uint32_t mask,
                         const uint8_t *const *arenas, uint8_t *residual, const cec_plan *plan,
                         void *stream) {
    if (int r = check_code(k, m, matrix)) return r;
    if (lid_self < k || lid_self >= k + m || !arenas || !residual || !plan)
        return fail(CEC_EINVAL, "cec_residual: bad args");
    if (int r = single_pattern_plan(plan, "cec_residual")) return r;
    int dev;
    if (int r = current_device(&dev)) return r;
    Streams st;
    Combo c;
    Combo::Out o{};
    o.stream = static_cast<uint8_t>(k + m);
    o.mode = kModeWrite;
    if (!arenas[lid_self]) return fail(CEC_EINVAL, "cec_residual: own parity arena is NULL");
    st.base[lid_self] = const_cast<uint8_t *>(arenas[lid_self]);
    c.in_stream[c.n_in] = static_cast<uint8_t>(lid_self);
    o.coef[c.n_in++] = 1;  // first touch copies the parity unit (recovery.c:79-82)
    for (int s = 0; s < k; ++s) {
        if (!(mask & (1u << s))) continue;
        if (!arenas[s]) return fail(CEC_EINVAL, "cec_residual: arena %d in mask is NULL", s);
        st.base[s] = const_cast<uint8_t *>(arenas[s]);
        c.in_stream[c.n_in] = static_cast<uint8_t>(s);
        o.coef[c.n_in++] = MATRIX(lid_self, s);  // recovery.c:91-93
    }
    st.base[k + m] = residual;
    c.outs.push_back(o);
    return run_combos(dev, st, {c}, plan, 0, static_cast<hipStream_t>(stream));
}

// Lost data lids and participating parity lids of a recovery mask, ascending
// (complete_recovery_bottom_half, memcached.c:7847-7894).
static int mask_split(int k, int m, uint32_t mask, int *lost, int *pars) {
    int n = 0, r = 0;
    for (int j = 0; j < k; ++j)
        if (!(mask & (1u << j))) lost[n++] = j;
    for (int p = k; p < k + m; ++p)
        if (mask & (1u << p)) pars[r++] = p;
    return n == r ? n : -1;
}

static int solve_inverse(int k, const int *matrix, int n, const int *lost, const int *pars,
                         int *inv) {
    int tmp[CEC_MAX_M * CEC_MAX_M];
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) tmp[r * n + c] = MATRIX(pars[r], lost[c]);
    return invert_matrix(tmp, inv, n);
}

CEC_API int cec_solve(int k, int m, const int *matrix, uint32_t mask,
                      const uint8_t *const *residuals, uint8_t *const *out, const cec_plan *plan,
                      void *stream) {
    if (int r = check_code(k, m, matrix)) return r;
    if (!mask_ok(k, m, mask) || !residuals || !out || !plan)
        return fail(CEC_EINVAL, "cec_solve: bad args (mask=0x%x)", mask);
    if (int r = single_pattern_plan(plan, "cec_solve")) return r;
    int dev;
    if (int r = current_device(&dev)) return r;
    int lost[CEC_MAX_K], pars[CEC_MAX_M], inv[CEC_MAX_M * CEC_MAX_M];
    const int n = mask_split(k, m, mask, lost, pars);
    if (n < 0) return fail(CEC_EINVAL, "cec_solve: mask 0x%x is not a recovery mask", mask);
    if (n == 0) return CEC_OK;
    if (solve_inverse(k, matrix, n, lost, pars, inv))
        return fail(CEC_ESINGULAR, "cec_solve: singular submatrix for mask 0x%x", mask);
    Streams st;
    Combo c;
    c.n_in = n;
    for (int r = 0; r < n; ++r) {
        if (!residuals[pars[r]]) return fail(CEC_EINVAL, "cec_solve: residual %d NULL", pars[r]);
        st.base[r] = const_cast<uint8_t *>(residuals[pars[r]]);
        c.in_stream[r] = static_cast<uint8_t>(r);
    }
    for (int x = 0; x < n; ++x) {
        if (!out[lost[x]]) return fail(CEC_EINVAL, "cec_solve: out[%d] NULL", lost[x]);
        st.base[CEC_MAX_M + x] = out[lost[x]];
        Combo::Out o{};
        o.stream = static_cast<uint8_t>(CEC_MAX_M + x);
        o.mode = kModeWrite;
        for (int r = 0; r < n; ++r) o.coef[r] = inv[x * n + r];  // memcached.c:7916-7922
        c.outs.push_back(o);
    }
    return run_combos(dev, st, {c}, plan, 0, static_cast<hipStream_t>(stream));
}

CEC_API int cec_decode(int k, int m, const int *matrix, const uint32_t *masks, int n_masks,
                       const uint8_t *const *arenas, uint8_t *const *out, const cec_plan *plan,
                       void *stream) {
    if (int r = check_code(k, m, matrix)) return r;
    if (!masks || n_masks < 1 || !arenas || !out || !plan)
        return fail(CEC_EINVAL, "cec_decode: bad args");
    int dev;
    if (int r = current_device(&dev)) return r;
    if (plan->n_ext && plan->max_pattern >= static_cast<uint32_t>(n_masks))
        return fail(CEC_EINVAL, "cec_decode: an extent names mask %u of %d", plan->max_pattern, n_masks);
    Streams st;
    for (int lid = 0; lid < k + m; ++lid) st.base[lid] = const_cast<uint8_t *>(arenas[lid]);
    for (int j = 0; j < k; ++j) st.base[k + m + j] = out[j];
    std::vector<Combo> combos(n_masks);
    for (int q = 0; q < n_masks; ++q) {
        const uint32_t mask = masks[q];
        if (!mask_ok(k, m, mask)) return fail(CEC_EINVAL, "cec_decode: bad mask 0x%x", mask);
        int lost[CEC_MAX_K], pars[CEC_MAX_M], inv[CEC_MAX_M * CEC_MAX_M];
        const int n = mask_split(k, m, mask, lost, pars);
        if (n < 0) return fail(CEC_EINVAL, "cec_decode: mask 0x%x is not a recovery mask", mask);
        if (n > 0 && solve_inverse(k, matrix, n, lost, pars, inv))
            return fail(CEC_ESINGULAR, "cec_decode: singular submatrix for mask 0x%x", mask);
        Combo &c = combos[q];
        // inputs: the n participating parities, then the k-n surviving data shards
        int surv[CEC_MAX_K], ns = 0;
        for (int j = 0; j < k; ++j)
            if (mask & (1u << j)) surv[ns++] = j;
        for (int r = 0; r < n; ++r) c.in_stream[c.n_in++] = static_cast<uint8_t>(pars[r]);
        for (int s = 0; s < ns; ++s) c.in_stream[c.n_in++] = static_cast<uint8_t>(surv[s]);
        for (int i = 0; i < c.n_in; ++i)
            if (!arenas[c.in_stream[i]])
                return fail(CEC_EINVAL, "cec_decode: arena %d (in mask 0x%x) is NULL",
                            c.in_stream[i], mask);
        // D_lost[x] = sum_r inv[x][r] * (P_r ^ sum_s MATRIX(P_r, s) * D_s)
        for (int x = 0; x < n; ++x) {
            if (!out[lost[x]]) return fail(CEC_EINVAL, "cec_decode: out[%d] is NULL", lost[x]);
            Combo::Out o{};
            o.stream = static_cast<uint8_t>(k + m + lost[x]);
            o.mode = kModeWrite;
            for (int r = 0; r < n; ++r) o.coef[r] = inv[x * n + r];
            for (int s = 0; s < ns; ++s) {
                int acc = 0;
                for (int r = 0; r < n; ++r) acc ^= gf_mul(inv[x * n + r], MATRIX(pars[r], surv[s]));
                o.coef[n + s] = acc;
            }
            c.outs.push_back(o);
        }
    }
    // AUTO: values of 64 KiB and more (large_values) run the LDS engine, ahead of PERM by a
    // median 3 % there (rotating or one mask: configs[4]'s 1 MiB D1-by-P1 rebuild +4.9 %);
    // 4 KiB values run PERM (rotating masks -1.7 %, one mask +1.1 %: within 2 %)
    return run_combos(dev, st, combos, plan, 0, static_cast<hipStream_t>(stream), nullptr,
                      large_values(plan));
}

CEC_API uint32_t cec_recovery_mask(int k, int m, int leader_lid, const int *connected) {
    if (k < 1 || m < 1 || k + m > 32 || !connected || leader_lid < 0 || leader_lid >= k + m)
        return 0;
    int remaining = k - 1;
    uint32_t mask = 1u << leader_lid;
    for (int i = 0; i < k + m && remaining; ++i) {
        if (i == leader_lid || !connected[i]) continue;
        mask |= 1u << i;
        --remaining;
    }
    return remaining ? 0u : mask;
}

// ============================================================== fast stream wait
// One lane stores v into mapped pinned memory once every earlier op on the stream has
// finished (stream order).
__global__ void cec_signal_kernel(uint32_t *flag, uint32_t v) {
    __threadfence_system();
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

namespace {
struct SignalCtx {  // per thread and device: a mapped pinned completion word
    int device = -1;
    uint32_t *flag = nullptr, *flag_dev = nullptr;
    uint32_t seq = 0;
    hipEvent_t fence = nullptr;  // recorded before the signal: a system-scope release
    ~SignalCtx() {  // (idle: every wait completed before its call returned)
        map_cache().release(device, flag, 64);
        if (fence) (void)hipEventDestroy(fence);
    }
};
thread_local SignalCtx t_signal;
}  // namespace

// Wait for everything enqueued on stream s, for the synchronous calls whose cost is
// their latency (the per-call drop-in, per-SET recovery folds).  A one-lane kernel
// writes a sequence number into mapped pinned memory behind the work and the host
// spins on it: 6.3 us per empty call against 10.5 us for hipStreamSynchronize
// (tools/launch_latency.hip, archive/profiles/r01_launch_latency.txt).  After 200 us (a large
// op, or a kernel that faulted and never signals) it falls back to
// hipStreamSynchronize, which also reports errors.
// `host_results`: the work wrote host-visible memory that the caller reads on return;
// `waves_released`: every wave that wrote it ended with its own system-scope release
// (kFlagSysRelease).  The completion is recorded for cec_last_sync.
thread_local cec_sync_record t_last_sync = {0, 0, 0, 0};

static int stream_wait(hipStream_t s, bool host_results, bool waves_released = false) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    SignalCtx &c = t_signal;
    if (c.device != dev) {
        map_cache().release(c.device, c.flag, 64);
        c.flag = c.flag_dev = nullptr;
        c.flag = static_cast<uint32_t *>(map_cache().acquire(dev, 64));
        if (!c.flag) return fail(CEC_ENOMEM, "completion flag");
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&c.flag_dev), c.flag, 0));
        __atomic_store_n(c.flag, 0u, __ATOMIC_RELEASE);
        c.seq = 0;
        if (c.fence) (void)hipEventDestroy(c.fence);
        c.fence = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&c.fence, hipEventDisableTiming));
        c.device = dev;
    }
    const uint32_t v = ++c.seq;
    const bool fence = host_results && !waves_released;
    t_last_sync.seq += 1;
    t_last_sync.host_results = host_results;
    t_last_sync.waves_released = host_results && waves_released;
    t_last_sync.fenced = fence;
    // The op's stores into host memory may still sit in the L2 of the XCDs its
    // workgroups ran on, and the signal kernel's own fence writes back only its XCD's
    // (a 4098-byte drop-in call read back its second tile stale on some boxes).  Either
    // every wave of the op ended with a system-scope release (kFlagSysRelease: the
    // drop-in), or an event recorded here with the system fence makes the command
    // processor write every L2 back before the signal kernel starts (4-5 us more per
    // call on one box, archive/profiles/r02_evidence_s3/fence_cost_ab.jsonl).  (Spinning on
    // hipEventQuery of that event instead of the signal kernel's flag measured the same
    // per call: archive/profiles/r02_evidence_s3/wait_mode_ab.jsonl.)
    if (fence) HIP_TRY(hipEventRecord(c.fence, s));
    hipLaunchKernelGGL(cec_signal_kernel, dim3(1), dim3(1), 0, s, c.flag_dev, v);
    HIP_TRY(hipGetLastError());
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(c.flag, __ATOMIC_ACQUIRE) == v) return CEC_OK;
        __builtin_ia32_pause();
        if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200))
            break;
    }
    HIP_TRY(hipStreamSynchronize(s));
    return CEC_OK;
}

CEC_API int cec_last_sync(cec_sync_record *out) {
    if (!out) return fail(CEC_EINVAL, "cec_last_sync: out is NULL");
    *out = t_last_sync;
    return CEC_OK;
}

#include "cec_drain.inc"
#include "cec_recovery.inc"
#include "cec_pool.inc"
#include "cec_hostbatch.inc"

// ============================================================== events / streams
CEC_API int cec_event_create(void **ev) {
    if (!ev) return fail(CEC_EINVAL, "NULL");
    hipEvent_t e;
    // Timing events only: no system-scope fence at record (the default fence writes the
    // L2 back between launches, which lengthens the measured interval).
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    *ev = e;
    return CEC_OK;
}
CEC_API int cec_event_destroy(void *ev) {
    HIP_TRY(hipEventDestroy(static_cast<hipEvent_t>(ev)));
    return CEC_OK;
}
CEC_API int cec_event_record(void *ev, void *stream) {
    HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(stream)));
    return CEC_OK;
}
CEC_API int cec_event_elapsed_ms(void *a, void *b, float *ms) {
    HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(b)));
    HIP_TRY(hipEventElapsedTime(ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)));
    return CEC_OK;
}
CEC_API int cec_stream_synchronize(void *stream) {
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return CEC_OK;
}
CEC_API int cec_device_count(int *count) {
    if (!count) return fail(CEC_EINVAL, "cec_device_count: NULL");
    *count = 0;
    if (hipGetDeviceCount(count) != hipSuccess) {
        (void)hipGetLastError();
        *count = 0;
    }
    return CEC_OK;
}
CEC_API int cec_set_device(int device) {
    HIP_TRY(hipSetDevice(device));
    int dev;
    return current_device(&dev);
}
CEC_API int cec_stream_create(void **stream) {
    if (!stream) return fail(CEC_EINVAL, "cec_stream_create: NULL");
    hipStream_t s;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return CEC_OK;
}
CEC_API int cec_stream_destroy(void *stream) {
    HIP_TRY(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return CEC_OK;
}
CEC_API int cec_copy(void *dst, const void *src, size_t n, void *stream) {
    if (n && (!dst || !src)) return fail(CEC_EINVAL, "cec_copy: NULL pointer");
    int dev;
    if (int r = current_device(&dev)) return r;
    if (n) HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
    return CEC_OK;
}

CEC_API int cec_host_register(void *p, size_t bytes, uint8_t **device_alias) {
    if (!p || !bytes || !device_alias) return fail(CEC_EINVAL, "cec_host_register: bad args");
    *device_alias = nullptr;
    int dev;
    if (int r = current_device(&dev)) return r;
    HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterMapped));
    void *d = nullptr;
    if (hipError_t e = hipHostGetDevicePointer(&d, p, 0); e != hipSuccess) {
        (void)hipHostUnregister(p);
        return fail(CEC_EHIP, "cec_host_register: hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    *device_alias = static_cast<uint8_t *>(d);
    host_region_add(p, bytes, *device_alias, dev);  // (the host batch reads bases there in place)
    return CEC_OK;
}

CEC_API int cec_host_unregister(void *p) {
    if (!p) return fail(CEC_EINVAL, "cec_host_unregister: NULL");
    int dev;
    if (int r = current_device(&dev)) return r;
    host_region_remove(p);
    HIP_TRY(hipHostUnregister(p));
    return CEC_OK;
}

// ============================================================== Jerasure drop-in
CEC_API int galois_single_multiply(int a, int b, int w) {
    if (w != 8) die("galois_single_multiply: only w = 8 is provided");
    return gf_mul(a, b);
}
CEC_API int galois_single_divide(int a, int b, int w) {
    if (w != 8) die("galois_single_divide: only w = 8 is provided");
    if ((b & 0xFF) == 0) return -1;
    return gf_div(a, b);
}
CEC_API int galois_inverse(int x, int w) { return galois_single_divide(1, x, w); }

CEC_API int *reed_sol_extended_vandermonde_matrix(int rows, int cols, int w) {
    if (w != 8 || rows < 1 || cols < 1 || rows > 256 || cols > 256) return nullptr;
    int *v = static_cast<int *>(calloc(static_cast<size_t>(rows) * cols, sizeof(int)));
    if (!v) return nullptr;
    v[0] = 1;
    if (rows == 1) return v;
    v[rows * cols - 1] = 1;
    for (int r = 1; r + 1 < rows; ++r)
        for (int c = 0, x = 1; c < cols; ++c, x = gf_mul(x, r)) v[r * cols + c] = x;
    return v;
}

CEC_API int *reed_sol_big_vandermonde_distribution_matrix(int rows, int cols, int w) {
    if (cols >= rows) return nullptr;
    int *m = reed_sol_extended_vandermonde_matrix(rows, cols, w);
    if (!m) return nullptr;
    auto at = [&](int r, int c) -> int & { return m[r * cols + c]; };
    for (int i = 1; i < cols; ++i) {  // column-reduce the top block to identity
        int r = i;
        while (r < rows && at(r, i) == 0) ++r;
        if (r == rows) { free(m); return nullptr; }
        if (r != i)
            for (int c = 0; c < cols; ++c) std::swap(at(r, c), at(i, c));
        if (at(i, i) != 1) {
            const int s = gf_inv(at(i, i));
            for (int q = 0; q < rows; ++q) at(q, i) = gf_mul(s, at(q, i));
        }
        for (int c = 0; c < cols; ++c) {
            const int e = at(i, c);
            if (c != i && e)
                for (int q = 0; q < rows; ++q) at(q, c) ^= gf_mul(e, at(q, i));
        }
    }
    for (int c = 0; c < cols; ++c) {  // first parity row -> all ones
        const int e = at(cols, c);
        if (e != 1) {
            const int s = gf_inv(e);
            for (int q = cols; q < rows; ++q) at(q, c) = gf_mul(s, at(q, c));
        }
    }
    for (int q = cols + 1; q < rows; ++q) {  // first column of later parity rows -> one
        const int e = at(q, 0);
        if (e != 1) {
            const int s = gf_inv(e);
            for (int c = 0; c < cols; ++c) at(q, c) = gf_mul(at(q, c), s);
        }
    }
    return m;
}

CEC_API int jerasure_invert_matrix(int *mat, int *inv, int rows, int w) {
    if (w != 8) {
        fprintf(stderr, "libcocytus_ec: jerasure_invert_matrix: only w = 8 is provided\n");
        return -1;
    }
    if (!mat || !inv || rows < 1) return -1;
    return invert_matrix(mat, inv, rows);
}

CEC_API int *jerasure_matrix_multiply(int *m1, int *m2, int r1, int c1, int r2, int c2, int w) {
    if (w != 8 || c1 != r2 || r1 < 1 || c2 < 1) return nullptr;
    int *p = static_cast<int *>(calloc(static_cast<size_t>(r1) * c2, sizeof(int)));
    if (!p) return nullptr;
    for (int i = 0; i < r1; ++i)
        for (int j = 0; j < c2; ++j) {
            int acc = 0;
            for (int x = 0; x < c1; ++x) acc ^= gf_mul(m1[i * c1 + x], m2[x * c2 + j]);
            p[i * c2 + j] = acc;
        }
    return p;
}

// Per-thread context of the synchronous drop-in: a stream and device staging.
namespace {
struct DropInCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t *dsrc = nullptr, *ddst = nullptr;
    size_t cap = 0;
    uint8_t *zc = nullptr;  // mapped pinned buffer (2 x zc_cap) for zero-copy calls
    void *zc_dev = nullptr;  // its device address
    size_t zc_cap = 0;
    ~DropInCtx() {
        if (stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        release();
    }
    // Buffers back to the process caches (idle: every call completed before returning);
    // freeing them would wait for the whole device.
    void release() {
        dev_cache().release(device, dsrc, cap);
        dev_cache().release(device, ddst, cap);
        map_cache().release(device, zc, 2 * zc_cap);
        dsrc = ddst = zc = nullptr;
        zc_dev = nullptr;
        cap = zc_cap = 0;
    }
};
thread_local DropInCtx t_ctx;
constexpr size_t kStageChunk = size_t(64) << 20;

// Pageable calls up to this size go zero-copy: the bytes are memcpy'd into a mapped
// pinned buffer and the kernel reads / writes it over PCIe, which saves the three DMA
// set-ups of the staged path (latency-bound at 4 KiB).  CEC_DROPIN_ZC_MAX overrides.
size_t zero_copy_max() {
    static const size_t v = [] {
        const char *e = getenv("CEC_DROPIN_ZC_MAX");
        return e ? static_cast<size_t>(strtoull(e, nullptr, 0)) : size_t(256) << 10;
    }();
    return v;
}

// Device-usable address for p, or NULL if p is pageable host memory; *host: the host
// may read p on return without a copy -- pinned host memory (the kernel reaches it over
// PCIe) or managed memory -- so a result written there needs the system-scope release.
void *device_view(void *p, bool *host) {
    *host = false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    *host = at.type == hipMemoryTypeHost || at.type == hipMemoryTypeManaged;
    if (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged ||
        at.type == hipMemoryTypeHost)
        return at.devicePointer;
    return nullptr;
}
}  // namespace

#define DROPIN_CHECK(expr)                                                                  \
    do {                                                                                    \
        int rc_ = (expr);                                                                   \
        if (rc_ != CEC_OK) {                                                                \
            char b_[640];                                                                   \
            snprintf(b_, sizeof b_, "galois_w08_region_multiply: %s", g_err);              \
            die(b_);                                                                        \
        }                                                                                   \
    } while (0)
#define DROPIN_HIP(expr)                                                                    \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            char b_[256];                                                                   \
            snprintf(b_, sizeof b_, "galois_w08_region_multiply: %s: %s", #expr,           \
                     hipGetErrorString(e_));                                                \
            die(b_);                                                                        \
        }                                                                                   \
    } while (0)

CEC_API void galois_w08_region_multiply(char *region, int multby, int nbytes, char *r2, int add) {
    if (multby < 0 || multby > 255) die("galois_w08_region_multiply: multby outside [0, 255]");
    if (nbytes <= 0) return;
    if (!region) die("galois_w08_region_multiply: region is NULL");
    if (r2 && add && multby == 0) return;
    int dev;
    DROPIN_CHECK(current_device(&dev));
    DropInCtx &c = t_ctx;
    if (c.device != dev) {
        if (c.stream) DROPIN_HIP(hipStreamDestroy(c.stream));
        c.stream = nullptr;
        c.release();  // (device addresses of the mapped buffer are per device)
        DROPIN_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        c.device = dev;
    }
    const size_t n = static_cast<size_t>(nbytes);
    char *dst = r2 ? r2 : region;
    const int mode_add = r2 ? add : 0;
    bool hs = false, hd = false;
    void *vs = device_view(region, &hs), *vd = device_view(dst, &hd);
    if (vs && vd) {  // device-resident (or pinned/mapped): run in place
        bool rel = false;  // (a host-visible destination: the kernel's waves release it themselves)
        DROPIN_CHECK(region_launch(dev, vs, multby, n, vd, mode_add, c.stream, true, hd ? kFlagSysRelease : 0, &rel));
        DROPIN_CHECK(stream_wait(c.stream, hd, rel));
        return;
    }
    const size_t n16 = (n + 15) & ~size_t(15);  // the kernel's extent in the staging
    const bool host_ok = (!vs || hs) && (!vd || hd);  // both reachable by the CPU's memcpy
    if (host_ok && n <= zero_copy_max()) {  // small host call: zero-copy through mapped pinned memory
        if (c.zc_cap < n16) {
            map_cache().release(dev, c.zc, 2 * c.zc_cap);
            c.zc_cap = std::max(n16, size_t(64) << 10);
            c.zc = static_cast<uint8_t *>(map_cache().acquire(dev, 2 * c.zc_cap));
            if (!c.zc) die("galois_w08_region_multiply: mapped staging allocation failed");
            DROPIN_HIP(hipHostGetDevicePointer(&c.zc_dev, c.zc, 0));
        }
        uint8_t *zs = c.zc, *zd = c.zc + c.zc_cap;
        memcpy(zs, region, n);
        if (mode_add) memcpy(zd, dst, n);
        uint8_t *ds = static_cast<uint8_t *>(c.zc_dev), *dd = ds + c.zc_cap;
        // n16 bytes: whole 16-byte chunks only, no byte scatter over PCIe (the padding's
        // results are not copied back)
        bool rel = false;
        DROPIN_CHECK(region_launch(dev, ds, multby, n16, dd, mode_add, c.stream, true, kFlagSysRelease, &rel));
        DROPIN_CHECK(stream_wait(c.stream, true, rel));  // (spinning on hipStreamQuery instead: no gain)
        memcpy(dst, zd, n);
        return;
    }
    // larger host buffers (or a device operand with a host result): stage through
    // device memory chunk by chunk
    const size_t want = std::min(n, kStageChunk);
    if (c.cap < want) {
        dev_cache().release(dev, c.dsrc, c.cap);
        dev_cache().release(dev, c.ddst, c.cap);
        c.dsrc = static_cast<uint8_t *>(dev_cache().acquire(dev, want));
        c.ddst = static_cast<uint8_t *>(dev_cache().acquire(dev, want));
        if (!c.dsrc || !c.ddst) die("galois_w08_region_multiply: device staging allocation failed");
        c.cap = want;
    }
    for (size_t o = 0; o < n; o += kStageChunk) {
        const size_t len = std::min(kStageChunk, n - o);
        DROPIN_HIP(hipMemcpyAsync(c.dsrc, region + o, len, hipMemcpyDefault, c.stream));
        if (mode_add)
            DROPIN_HIP(hipMemcpyAsync(c.ddst, dst + o, len, hipMemcpyDefault, c.stream));
        DROPIN_CHECK(region_launch(dev, c.dsrc, multby, len, c.ddst, mode_add, c.stream, true));
        DROPIN_HIP(hipMemcpyAsync(dst + o, c.ddst, len, hipMemcpyDefault, c.stream));
        DROPIN_HIP(hipStreamSynchronize(c.stream));
    }
    // (the result came back by DMA, complete and visible when the stream synchronised)
    t_last_sync.seq += 1;
    t_last_sync.host_results = !vd || hd;
    t_last_sync.waves_released = 0;
    t_last_sync.fenced = 1;
}
