// cec_kernels.hpp -- CDNA4 (gfx950) HIP kernels for Cocytus' erasure-coding hot path.
//
// Every op on the path -- galois_w08_region_multiply, the per-SET
// diff-update (a2 + a3 = a4), full-stripe encode (a5), the recovery residual (a6)
// and the leader solve (a7) -- is a GF(2^8) linear combination of byte streams
// taken at the same arena offset:
//
//     out[l][off .. off+len)  (^)=  sum_i  coef[l][i] * in[i][off .. off+len)
//
// so one kernel family implements all of them.  A launch walks a work-list of
// 4 KiB tiles (CEC_UNIT_SIZE, /root/reference/const.h:26) built from the batch's
// extents; each tile carries a pattern index that selects the inputs, outputs and
// coefficients (per source shard for diff-update, per erasure mask for decode).
//
// Hardware mapping (MI355X):
//   * one 16-byte chunk per lane: a 4 KiB tile is 256 lanes, as one 256-lane
//     workgroup or (full, line-aligned tiles) four one-wave workgroups of 64
//     (split_shift); every stream of a tile is read with one fully coalesced
//     global_load_dwordx4 per lane (uniform SGPR base + per-lane VGPR offset);
//   * tile metadata and coefficient tables are wave-uniform and live in SGPRs
//     (constant-address-space loads -> s_load);
//   * GF multiply by a uniform coefficient c on 4 packed bytes:
//       PERM engine: c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6], three v_perm_b32
//                    byte lookups per dword (tables are 8 bytes: two SGPRs);
//       LDS engine : 256-entry product rows c*x = exp[log x + log c], one per
//                    coefficient of the tile's pattern, built from the log / antilog
//                    tables and staged in LDS per workgroup: one ds_read_u8 per byte;
//     no MFMA: this is byte-field arithmetic, HBM-bound.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf256.hpp"

namespace cec {

constexpr int kTile = 4096;      // bytes per tile = kBlock lanes x 16 B
constexpr int kBlock = 256;
constexpr int kBlockLog2 = 8;
constexpr uint64_t kLineBytes = 128;  // L2 / HBM line
static_assert(kBlock == 1 << kBlockLog2, "kBlock must be a power of two");
constexpr int kMaxStreams = 48;  // 16 data + 8 parity + 16 recovered + staging/diff ...
constexpr int kPatN = 16;        // inputs per pattern (k <= CEC_MAX_K)
constexpr int kPatL = 4;         // outputs per launch pattern (host splits more)

enum : int32_t { kModeWrite = 0, kModeXor = 1 };

// One linear combination.  Lives in device memory and is read with scalar loads,
// so every field is 32-bit (gfx9 scalar loads are dword-granular).
struct alignas(16) Pattern {
    int32_t n_in;
    int32_t n_out;
    int32_t in_stream[kPatN];
    int32_t in_src[kPatN];        // 1: address with extent.src_off, 0: with extent.off
    int32_t out_stream[kPatL];
    int32_t out_src[kPatL];
    int32_t out_mode[kPatL];      // kModeWrite / kModeXor
    int32_t lds_rows;             // LDS engine: product rows this pattern stages ...
    int32_t lds_row_base;         // ... starting at row lds_row_base of CombineArgs::rows
    int32_t coef[kPatL][kPatN];
    uint32_t tab[kPatL][kPatN][5];  // PERM: PermTab; LDS: tab[..][0] = LDS byte offset of the row
};

// One tile of the work-list: a <= 4 KiB piece of one extent, same layout as
// cec_extent, so a tile is fetched with one scalar load and no indirection.
struct Tile {
    uint64_t off;      // arena offset of the piece
    uint64_t src_off;  // staging offset of the piece
    uint32_t len;      // 1 .. kTile
    uint32_t pattern;
};

// Kernel arguments with S stream slots.  Patterns name streams by slot.  The host
// writes a launch's whole kernarg segment for every dispatch, and 424 B of arguments
// cost 1.3 us more host time per launch than none (tools/dropin_breakdown.hip).  So a
// launch whose patterns use only slots 0 and 1 (region multiply, the drop-in) takes
// S = 2, and the kernel reads its grid size from here rather than from gridDim /
// blockDim: those come from the hidden arguments, which add 256 B to every segment.
// CombineArgsN::flags: every wave ends with a system-scope release (its XCD's L2 written
// back, its stores complete), for launches whose outputs the host reads on a signal
// that does not come from the runtime (the synchronous drop-in over host memory).
// Honoured by the 1 x 1 (region multiply) launches, which select the kSysRel kernel.
constexpr uint32_t kFlagSysRelease = 1u;
// CombineArgsN::flags: the wide stores write through the XCD's L2 (sc1) instead of
// non-temporal stores that keep the line there.  The host sets it for launches small
// enough that what they write is read again from the memory-side cache, or that the
// dirty lines they would leave in L2 are a visible part of the launch (DESIGN.md §4:
// the per-GPU shares of strong scaling).
constexpr uint32_t kFlagWriteThrough = 2u;

template <int S>
struct CombineArgsN {
    uint8_t *base[S];
    const Tile *tiles;       // NULL: implicit region [0, implicit_len), pattern 0
    const Pattern *patterns;
    const uint8_t *rows;     // LDS engine: 256-B product rows (c*x for x = 0..255)
    uint64_t implicit_len;
    uint32_t n_tiles;
    uint32_t split_shift;  // 2^split_shift workgroups of kBlock >> split_shift lanes per tile
    uint32_t grid;         // workgroups in the launch (the grid-stride step)
    uint32_t flags;        // kFlag* bits (fills the struct's padding)
};
using CombineArgs = CombineArgsN<kMaxStreams>;
constexpr int kNarrowStreams = 2;

#define CEC_CONST __attribute__((address_space(4)))
#define CEC_GLOBAL __attribute__((address_space(1)))

// Read-only kernel inputs are re-addressed in the constant address space so that
// wave-uniform loads of them become scalar (s_load) loads.
template <class T>
__device__ inline const CEC_CONST T *as_const(const T *p) {
    return (const CEC_CONST T *)(uintptr_t)p;
}

// Arena bytes: global address space, so a uniform base + per-lane offset becomes
// global_load_dwordx4 v, v_off, s[base] (no flat addressing, no 64-bit VGPR math).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streamed bytes are touched once per launch: non-temporal loads and stores (nt)
// measured +5-10 % over the default policy on this access pattern.
__device__ inline uint4 ld16(const uint8_t *base, uint32_t off) {
    const u32x4 v = __builtin_nontemporal_load((const CEC_GLOBAL u32x4 *)((uintptr_t)base + off));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ inline void st16(uint8_t *base, uint32_t off, const uint4 &v) {
    u32x4 w;
    w.x = v.x;
    w.y = v.y;
    w.z = v.z;
    w.w = v.w;
    __builtin_nontemporal_store(w, (CEC_GLOBAL u32x4 *)((uintptr_t)base + off));
}
// Write-through (sc1) store of one 16-B chunk at base + off, off < kTile: a buffer store
// through a descriptor built from the wave-uniform tile base (SGPRs).
__device__ inline void st16_wt(uint8_t *base, uint32_t off, const uint4 &v) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, kTile, 0x00020000);
    u32x4 w;
    w.x = v.x;
    w.y = v.y;
    w.z = v.z;
    w.w = v.w;
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, off, 0, 16 /* sc1 */);
}
__device__ inline uint32_t ld8(const uint8_t *base, uint32_t off) {
    return *(const CEC_GLOBAL uint8_t *)((uintptr_t)base + off);
}
__device__ inline void st8(uint8_t *base, uint32_t off, uint32_t v) {
    *(CEC_GLOBAL uint8_t *)((uintptr_t)base + off) = static_cast<uint8_t>(v);
}

// ---------------------------------------------------------------- engines
struct PermEngine {
    static constexpr bool kStaged = false;
    struct Sel {
        uint32_t s0, s1, s2;
    };
    __device__ static inline Sel sel(uint32_t x) {
        return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
    }
    __device__ static inline uint32_t mul(const Sel &s, const CEC_CONST uint32_t *t,
                                          const uint8_t *) {
        const uint32_t a = __builtin_amdgcn_perm(t[1], t[0], s.s0);
        const uint32_t b = __builtin_amdgcn_perm(t[3], t[2], s.s1);
        const uint32_t c = __builtin_amdgcn_perm(t[4], t[4], s.s2);
        return a ^ b ^ c;
    }
};

// One 256-B row per non-trivial coefficient of the tile's pattern, row_c[x] = c*x
// (row_c[0] = 0: no zero sentinel).  A ds_read_u8 of a 64-dword row has at most two
// distinct dwords per bank (32 banks for byte / dword reads), and lanes that hit the
// same dword broadcast, so a random lookup costs <= 2 LDS cycles per 32-lane group.
struct LdsEngine {
    static constexpr bool kStaged = true;
    struct Sel {
        uint32_t b0, b1, b2, b3;
    };
    __device__ static inline Sel sel(uint32_t x) {
        return Sel{x & 0xFFu, (x >> 8) & 0xFFu, (x >> 16) & 0xFFu, x >> 24};
    }
    __device__ static inline uint32_t mul(const Sel &s, const CEC_CONST uint32_t *t,
                                          const uint8_t *lds) {
        const uint8_t *row = lds + t[0];
        return static_cast<uint32_t>(row[s.b0]) | (static_cast<uint32_t>(row[s.b1]) << 8) |
               (static_cast<uint32_t>(row[s.b2]) << 16) | (static_cast<uint32_t>(row[s.b3]) << 24);
    }
};

// ---------------------------------------------------------------- helpers
struct TileRef {
    uint64_t off, src_off;
    uint32_t len;  // bytes of this tile, 1..kTile
    uint32_t pattern;
};

template <class A>
__device__ inline TileRef load_tile(const A &a, uint32_t t) {
    TileRef r;
    if (a.tiles == nullptr) {
        const uint64_t o = static_cast<uint64_t>(t) * kTile;
        const uint64_t rem = a.implicit_len - o;
        r.off = o;
        r.src_off = o;
        r.len = rem < kTile ? static_cast<uint32_t>(rem) : kTile;
        r.pattern = 0;
    } else {
        const CEC_CONST Tile *tl = as_const(a.tiles) + t;
        r.off = tl->off;
        r.src_off = tl->src_off;
        r.len = tl->len;
        r.pattern = tl->pattern;
    }
    return r;
}

// A ragged chunk: the first cnt (1..16) bytes at base+off.  Branch-free: byte b
// reads address off + min(b, cnt-1), so all 16 loads are in bounds and in flight
// together (one memory latency, not sixteen dependent ones); bytes >= cnt read 0.
__device__ inline uint4 gather16(const uint8_t *base, uint32_t off, uint32_t cnt) {
    uint32_t v[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) v[b] = ld8(base, off + min(static_cast<uint32_t>(b), cnt - 1));
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) w[b >> 2] |= (static_cast<uint32_t>(b) < cnt ? v[b] : 0u) << (8 * (b & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Store the first cnt bytes of v at base+off.  Byte b goes to off + min(b, cnt-1)
// with the value of that clamped byte, so surplus stores rewrite the last valid byte
// with its own (correct) value: no predication, never out of bounds.
__device__ inline void scatter16(uint8_t *base, uint32_t off, uint32_t cnt, const uint4 &v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        const uint32_t q = min(static_cast<uint32_t>(b), cnt - 1);
        st8(base, off + q, w[q >> 2] >> (8 * (q & 3)));
    }
}

// acc[l] ^= sum_i coef[l][i] * x[i] on one 16-byte chunk of every stream.
template <int NT, int LT, class Eng>
__device__ inline void compute_chunk(const CEC_CONST Pattern *P, int n_in, int n_out,
                                     const uint4 (&x)[NT], uint4 (&acc)[LT], const uint8_t *lds) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        if (i >= n_in) continue;
        const uint32_t xv[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
        typename Eng::Sel s[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) s[w] = Eng::sel(xv[w]);
#pragma unroll
        for (int l = 0; l < LT; ++l) {
            if (l >= n_out) continue;
            const int c = P->coef[l][i];
            if (c == 0) continue;
            if (c == 1) {
                acc[l].x ^= xv[0];
                acc[l].y ^= xv[1];
                acc[l].z ^= xv[2];
                acc[l].w ^= xv[3];
            } else {
                const CEC_CONST uint32_t *tb = P->tab[l][i];
                acc[l].x ^= Eng::mul(s[0], tb, lds);
                acc[l].y ^= Eng::mul(s[1], tb, lds);
                acc[l].z ^= Eng::mul(s[2], tb, lds);
                acc[l].w ^= Eng::mul(s[3], tb, lds);
            }
        }
    }
}

// ---------------------------------------------------------------- the kernel
// NT / LT: input / output counts.  kExact: the patterns have exactly NT inputs and
// LT outputs (the hot shapes: straight-line loads, no guards); otherwise NT / LT
// are capacities and the pattern's n_in / n_out are wave-uniform runtime counts.
// kAcc: which outputs are read-modify-write (XOR-accumulate):
//   0 none, 1 all, 2 all but the last (diff-update + install), 3 per pattern.
enum : int { kAccNone = 0, kAccAll = 1, kAccAllButLast = 2, kAccRuntime = 3 };

// A workgroup covers 1 / 2^split_shift of a tile (blockDim = kBlock >> split_shift):
// work item g is tile g >> split_shift, part g & (2^split_shift - 1).
// kSysRel: every wave ends with a system-scope release (kFlagSysRelease launches; a
// template parameter, so the batched kernels carry no epilogue at all).
// LDS engine, full aligned tiles: stage the product rows before the stream loads (the
// fast path in combine_kernel) for the diff-update shapes only (2 inputs, parity
// read-modify-write).  There it ran the diff-update + install 2.4 % faster; in the
// encode (3 x 2) the second path's registers cost SGPR spills and occupancy (+10 %),
// and the fixed-mask decode / residual (3 x 1) lost 2-3 %
// (profiles/r03_evidence/lds_early_rows/).
template <int NT, int kAcc, bool kExact>
constexpr bool kEarlyRows = kExact && NT == 2 && (kAcc == kAccAll || kAcc == kAccAllButLast);

template <int NT, int LT, class Eng, int kAcc, bool kExact, int S = kMaxStreams, bool kSysRel = false>
__global__ __launch_bounds__(kBlock) void combine_kernel(CombineArgsN<S> a) {
    extern __shared__ uint4 cec_lds_rows[];  // LDS engine: the pattern's product rows
    const uint8_t *lds = reinterpret_cast<const uint8_t *>(cec_lds_rows);
    const uint32_t sh = a.split_shift;
    const uint64_t n_work = static_cast<uint64_t>(a.n_tiles) << sh;

    // The LDS engine keeps the hardware grid / workgroup sizes: with them its register
    // allocation holds the step in a register, while a.grid was re-loaded (with a full
    // scalar wait) at the end of every tile, 3 % slower on the encode (tools/track_ab.sh).
    const uint32_t step = Eng::kStaged ? gridDim.x : a.grid;
    for (uint64_t g = blockIdx.x; g < n_work; g += step) {
        const uint32_t t = static_cast<uint32_t>(g >> sh);
        const uint32_t part = static_cast<uint32_t>(g) & ((1u << sh) - 1u);
        const uint32_t lane = (part << (kBlockLog2 - sh)) + threadIdx.x;
        const TileRef tr = load_tile(a, t);
        const CEC_CONST Pattern *P = as_const(a.patterns) + tr.pattern;
        const int n_in = kExact ? NT : P->n_in;
        const int n_out = kExact ? LT : P->n_out;
        if (!kExact && n_out == 0) continue;
        // A workgroup that walks several tiles (a launch past one dispatch's 2^32 - 1
        // work items) must not re-stage LDS rows while lanes still read the previous tile's.
        if constexpr (Eng::kStaged)
            if (g != blockIdx.x) __syncthreads();
        auto is_acc = [&](int l) -> bool {
            if constexpr (kAcc == kAccNone) return false;
            else if constexpr (kAcc == kAccAll) return true;
            else if constexpr (kAcc == kAccAllButLast) return l < LT - 1;
            else return P->out_mode[l] == kModeXor;
        };

        const uint8_t *in[NT];
        uint8_t *out[LT];
        uint64_t mis = 0;
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            in[i] = nullptr;
            if (i < n_in) {
                in[i] = a.base[P->in_stream[i]] + (P->in_src[i] ? tr.src_off : tr.off);
                mis |= reinterpret_cast<uint64_t>(in[i]);
            }
        }
#pragma unroll
        for (int l = 0; l < LT; ++l) {
            out[l] = nullptr;
            if (l < n_out) {
                out[l] = a.base[P->out_stream[l]] + (P->out_src[l] ? tr.src_off : tr.off);
                mis |= reinterpret_cast<uint64_t>(out[l]);
            }
        }

        // one 16-byte chunk per lane; the value's ragged tail (len = vlen + 2 is
        // rarely a multiple of 16) and tiles of misaligned device pointers use the
        // branch-free byte gather / scatter, everything else dwordx4.
        const uint32_t pos = lane * 16;
        if constexpr (Eng::kStaged && kEarlyRows<NT, kAcc, kExact>) {
            if ((mis & 15) == 0 && tr.len == kTile) {
                // A full, aligned tile (wave-uniform: every lane one whole chunk), the
                // LDS engine's common case.  Its product rows are fetched BEFORE the
                // stream loads, and the stream loads are unconditional, so the LDS write
                // waits only for the rows (vmcnt counts loads in order) and the write
                // and the barrier complete under the streams' HBM latency; the lookups
                // start as soon as the stream data lands.  (Staged after the stream
                // loads, below, the write waits for every stream load.)
                const uint32_t nb16 = static_cast<uint32_t>(P->lds_rows) * 16u;
                const uint4 *row_src = reinterpret_cast<const uint4 *>(a.rows) + P->lds_row_base * 16;
                uint4 row0 = make_uint4(0, 0, 0, 0);
                if (threadIdx.x < nb16) row0 = row_src[threadIdx.x];
                uint4 x[NT];
                uint4 acc[LT];
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    if (i < n_in) x[i] = ld16(in[i], pos);
#pragma unroll
                for (int l = 0; l < LT; ++l) {
                    acc[l] = make_uint4(0, 0, 0, 0);
                    if (l < n_out && is_acc(l)) acc[l] = ld16(out[l], pos);
                }
                if (nb16) {
                    if (threadIdx.x < nb16) cec_lds_rows[threadIdx.x] = row0;
                    for (uint32_t b = threadIdx.x + blockDim.x; b < nb16; b += blockDim.x)
                        cec_lds_rows[b] = row_src[b];  // (more rows than lanes)
                    __syncthreads();
                }
                compute_chunk<NT, LT, Eng>(P, n_in, n_out, x, acc, lds);
#pragma unroll
                for (int l = 0; l < LT; ++l)
                    if (l < n_out) st16(out[l], pos, acc[l]);
                continue;
            }
        }
        const bool active = pos < tr.len;
        if constexpr (!Eng::kStaged)
            if (!active) continue;  // (staged engines keep every lane to the barrier)
        const uint32_t cnt = active ? min(16u, tr.len - pos) : 16u;
        const bool wide = (mis & 15) == 0 && cnt == 16;
        uint4 x[NT];
        uint4 acc[LT];
        if (!active) {
        } else if (wide) {
#pragma unroll
            for (int i = 0; i < NT; ++i)
                if (i < n_in) x[i] = ld16(in[i], pos);
#pragma unroll
            for (int l = 0; l < LT; ++l) {
                acc[l] = make_uint4(0, 0, 0, 0);
                if (l < n_out && is_acc(l)) acc[l] = ld16(out[l], pos);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NT; ++i)
                if (i < n_in) x[i] = gather16(in[i], pos, cnt);
#pragma unroll
            for (int l = 0; l < LT; ++l) {
                acc[l] = make_uint4(0, 0, 0, 0);
                if (l < n_out && is_acc(l)) acc[l] = gather16(out[l], pos, cnt);
            }
        }
        if constexpr (Eng::kStaged) {
            // Stage this pattern's product rows (L2-resident, 256 B each; 512 B for an
            // RS(3,2) encode) while the stream loads above are in flight.
            // A pattern of XORs only (coefficients 0 / 1: e.g. every decode led by the
            // all-ones parity row) has no rows and skips the barrier; the branch is
            // uniform over the workgroup (one tile, one pattern).
            const uint32_t nb = static_cast<uint32_t>(P->lds_rows) * 256u;
            if (nb) {
                const uint4 *src = reinterpret_cast<const uint4 *>(a.rows) + P->lds_row_base * 16;
                for (uint32_t b = threadIdx.x; b < nb / 16; b += blockDim.x) cec_lds_rows[b] = src[b];
                __syncthreads();
            }
            if (!active) continue;
        }
        compute_chunk<NT, LT, Eng>(P, n_in, n_out, x, acc, lds);
        if (wide) {
            // (the LDS engine keeps non-temporal stores: the branch alone cost its encode
            // 1 %, profiles/r03_evidence/lds_engine_ab/)
            if (!Eng::kStaged && (a.flags & kFlagWriteThrough)) {
#pragma unroll
                for (int l = 0; l < LT; ++l)
                    if (l < n_out) st16_wt(out[l], pos, acc[l]);
            } else {
#pragma unroll
                for (int l = 0; l < LT; ++l)
                    if (l < n_out) st16(out[l], pos, acc[l]);
            }
        } else {
#pragma unroll
            for (int l = 0; l < LT; ++l)
                if (l < n_out) scatter16(out[l], pos, cnt, acc[l]);
        }
    }
    if constexpr (kSysRel) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this XCD's L2 written back
        // ... and completed before the wave ends (the fence alone leaves the wait to a
        // following store, and there is none)
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

}  // namespace cec
