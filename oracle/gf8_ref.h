/*
 * oracle/gf8_ref.h -- CPU restatement of Cocytus' erasure-coding hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (cocytus_amd/, include/)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / the timed CPU
 * baseline, never as the thing measured or shipped.
 *
 * PARITY UNPINNED: the reference's arithmetic lives in Jerasure 2.x +
 * GF-Complete (linked as -lJerasure, /root/reference/Makefile.am:46,49), which
 * is neither vendored in /root/reference nor installed in this image, and the
 * reference's own tests (t/ *.t, testapp.c) hold no parity / decode / matrix
 * vectors.  This file restates the published Jerasure 2.x
 * / GF-Complete semantics the call sites rely on; it is cross-checked against
 * independent known answers (carry-less GF(2^8) arithmetic in pure Python,
 * SURVEY.md §8c restated matrices, algebraic invariants), not against the
 * reference binary.
 *
 * Field: GF(2^8), primitive polynomial x^8+x^4+x^3+x^2+1 (0x11D; Jerasure's
 * prim_poly[8] = 0435 octal; GF-Complete's w=8 default), generator 2.
 */
#ifndef COCYTUS_ORACLE_GF8_REF_H
#define COCYTUS_ORACLE_GF8_REF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scalar field (Jerasure galois_single_multiply / galois_single_divide, w=8) ---- */
int ref_gf_mul(int a, int b);
int ref_gf_div(int a, int b);          /* a / b; returns -1 if b == 0 (Jerasure convention) */
int ref_gf_exp(int i);                 /* 2^i, i in [0, 255) */
int ref_gf_log(int a);                 /* log2(a), a in [1, 256) */

/* ---- region multiply: galois_w08_region_multiply(region, multby, nbytes, r2, add) ----
 * add != 0:  r2[i] ^= multby * region[i]   (every Cocytus call site passes add = 1)
 * add == 0:  r2[i]  = multby * region[i]
 * r2 == NULL: region[i] = multby * region[i]  (Jerasure 1.x documented in-place form)
 * Scalar, byte at a time: the semantic definition.                              */
void ref_region_multiply(uint8_t *region, int multby, long nbytes, uint8_t *r2, int add);

/* ---- coding matrix: reed_sol_big_vandermonde_distribution_matrix(rows, cols, 8) ----
 * Called as (K+M, K, 8) at memcached.c:6845.  Returns malloc'd rows*cols ints
 * (row-major, MATRIX(x,y) = m[x*K+y], memcached.h:52) or NULL on bad args.      */
int *ref_extended_vandermonde(int rows, int cols);
int *ref_big_vandermonde(int rows, int cols);

/* ---- jerasure_invert_matrix(mat, inv, rows, 8): Gauss-Jordan; clobbers mat;
 * returns 0, or -1 if singular (memcached.c:7907-7908 asserts 0).                */
int ref_invert_matrix(int *mat, int *inv, int rows);

/* ---- the hot-path chains, restated call for call ---- */

/* memcached.c:2673-2681 (and the substitute twin :5602-5611):
 * diff = new; galois_w08_region_multiply(old, 1, n, diff, 1)  =>  diff = new ^ old */
void ref_set_diff(const uint8_t *oldv, const uint8_t *newv, long n, uint8_t *diff);

/* memcached.c:7762-7767 (process_rep_command on parity lid_self):
 * galois_w08_region_multiply(diff, MATRIX(lid_self, lid_src), n, parity, 1)        */
void ref_parity_apply(const int *matrix, int k, int lid_self, int lid_src,
                      const uint8_t *diff, long n, uint8_t *parity);

/* The per-SET diff-update as the cluster runs it: the data
 * server computes the diff, each of the M parities applies its own row, the data
 * server installs the new value (memcached.c:5666) when install != 0.           */
void ref_diff_update(const int *matrix, int k, int m, int shard_j,
                     uint8_t *old_in_arena, const uint8_t *newv, long n,
                     uint8_t *const *parity, int install);

/* Full-stripe encode as K successive SETs into zero parity:
 * P_p = sum_j MATRIX(K+p, j) * D_j, chained one galois_w08_region_multiply per
 * (p, j) exactly like K SETs with old = 0.                                       */
void ref_encode(const int *matrix, int k, int m, const uint8_t *const *data,
                uint8_t *const *parity, long n);

/* start_recovery's participant mask (memcached.c:8136-8151): the leader plus the
 * first K-1 connected lids in ascending order.  connected[lid] != 0 if peer is
 * connected (the leader's own entry is ignored).  Returns 0 if not enough.      */
uint32_t ref_recovery_mask(int k, int m, int leader_lid, const int *connected);

/* recovery_recover_units (recovery.c:61-96) for one parity lid_self over a range
 * of units: on first touch copy the parity unit, then XOR in MATRIX(self, peer) *
 * survivor unit.  Restated for one contiguous range: residual must be n bytes,
 * touched is the unit's update flag (0 = first touch).                           */
void ref_recover_units(const int *matrix, int k, int lid_self, int peer_lid,
                       const uint8_t *own_parity, const uint8_t *peer_data, long n,
                       uint8_t *residual, int *touched);

/* recovery_try_update_unit (recovery.c:99-131) arithmetic: a write landing during
 * recovery folds MATRIX(self, peer) * diff into the in-flight residual at offset. */
void ref_try_update_unit(const int *matrix, int k, int lid_self, int peer_lid,
                         const uint8_t *diff, long len, uint8_t *residual_at_offset);

/* complete_recovery_bottom_half arithmetic (memcached.c:7842-7922): given the
 * residuals C[x] of the participating parities (ascending lid), solve
 * data[i] = sum_j inv[i][j] * C[j] over nbuf bytes; out[i] is the i-th lost data
 * shard (ascending lid).  Returns n_lost, or -1 if the submatrix is singular.    */
int ref_bottom_half(const int *matrix, int k, int m, uint32_t mask,
                    const uint8_t *const *C, long nbuf, uint8_t *const *out);

/* Whole online-recovery chain for one range: residual on every participating
 * parity from the surviving data in mask (recover_units_reply order = ascending
 * lid), then the leader's bottom half.  arenas[lid] = that lid's bytes for the
 * range (lost ones may be NULL); out[i] = i-th lost data shard.  Returns n_lost. */
int ref_decode(const int *matrix, int k, int m, uint32_t mask,
               const uint8_t *const *arenas, long n, uint8_t *const *out);

/* ---- CPU baseline (cpu_baseline leg of bench.py only) ----
 * GF-Complete's default w=8 region kernel restated: SPLIT(8,4) split-nibble
 * tables looked up 32 bytes at a time with AVX2 vpshufb (GF-Complete uses the
 * 16-byte SSSE3 form).  r2 ^= c * region.                                        */
void ref_region_multiply_simd(const uint8_t *region, int multby, long nbytes, uint8_t *r2);
int ref_simd_available(void);

/* Threaded CPU baseline over a batch of stripes, chained as the reference does
 * (one region multiply per (parity, shard) for encode; residual + bottom half for
 * decode).  Returns elapsed seconds (CLOCK_MONOTONIC) for `reps` passes.         */
double ref_bench_encode_decode(int k, int m, long n, long nstripes, int threads,
                               int reps, int do_decode);
/* The same batch filled once, then `samples` timed passes of `reps` repetitions:
 * t[i] = seconds of pass i (the first is the caller's warm-up). 0, or -1 on bad args. */
int ref_bench_encode_decode_samples(int k, int m, long n, long nstripes, int threads,
                                    int reps, int do_decode, int samples, double *t);
/* The same with per-stripe lengths lens[s] (mixed value sizes, SURVEY §8d cfg 3), packed
 * at 16-B aligned offsets as ecalloc.c:176 places them; threads split by bytes.  lens ==
 * NULL is the uniform-n form above. */
int ref_bench_encode_decode_sizes(int k, int m, long n, const long *lens, long nstripes, int threads,
                                  int reps, int do_decode, int samples, double *t);

/* The parity's drain loop as the reference runs it (one thread, memcached.c:4350 ->
 * process_rep_command -> galois_w08_region_multiply(diff, MATRIX(self, lid), n,
 * parity + addr, 1) per pending diff): diffs packed at offsets soffs[i].  Returns
 * elapsed seconds (CLOCK_MONOTONIC). */
double ref_bench_apply(const uint8_t *stage, const uint64_t *soffs, const uint64_t *addrs,
                       const uint32_t *lens, const int *coefs, int n, uint8_t *parity);

/* One parity's online recovery of a single lost data shard over nbuf bytes as the
 * reference runs it (one thread): per peer message, per 4 KiB unit, first touch copies
 * the parity unit then region-multiplies the peer unit in (recovery.c:72-94); then the
 * leader's bottom half into a zeroed buffer (memcached.c:7913-7922).  Seconds. */
double ref_bench_recover(const uint8_t *parity, const uint8_t *const *peers, const int *coefs,
                         int npeers, int inv, long nbuf, uint8_t *residual, uint8_t *out);

/* A data process's SET diffs as the reference computes them (one thread, complete_nread,
 * memcached.c:2676-2681): per SET, diff = value (memcpy), then diff ^= 1 * ecmem[addr]
 * (galois_w08_region_multiply).  Value i at values + voffs[i], diff i at diffs + doffs[i].
 * Seconds. */
double ref_bench_set_diffs(const uint8_t *values, const uint64_t *voffs, const uint8_t *ecmem,
                           const uint64_t *addrs, const uint32_t *lens, int n, uint8_t *diffs,
                           const uint64_t *doffs);

/* A parity leading the recovery of nreq requests of `units` 4 KiB units each (request q:
 * units starts[q] .. starts[q] + units - 1 of ecmem), a single lost data shard, as the
 * reference runs it on one thread: per reply (replies[q * npeers + p], coefficient
 * coefs[p]) and per unit, recovery_recover_units (recovery.c:72-94: first touch mallocs the
 * unit and copies the parity unit in, then the peer unit is region-multiplied in); then per
 * request the bottom half (memcached.c:7853-7922: the units copied into one buffer, a
 * calloc'd output, output ^= inv * buffer).  outs[q] (units * 4096 bytes) receive the
 * rebuilt bytes after the clock stops.  Seconds. */
double ref_bench_recover_requests(const uint8_t *ecmem, const int *starts, int nreq, int units,
                                  const uint8_t *const *replies, int npeers, const int *coefs, int inv,
                                  uint8_t *const *outs);

#ifdef __cplusplus
}
#endif
#endif
