/*
 * cocytus_ec.h -- batched, device-resident erasure-coding API of libcocytus_ec.so
 * (MI355X / gfx950, hand-written HIP kernels; no MFMA, no Jerasure).
 *
 * This is the additive entry-point set SURVEY.md §8(b) asks for next to the three
 * drop-in Jerasure symbols (galois.h / jerasure.h / reed_sol.h).  Every call is
 * asynchronous on the given HIP stream (NULL = the default stream), takes device
 * pointers only, and returns a cec_status.  Nothing here falls back to the CPU:
 * a missing GPU is CEC_ENODEV.
 *
 * Layout contract (Cocytus): every data shard j and every parity p owns an arena
 * (ecmem, /root/reference/ecmem.h:29-58).  A value is the byte range
 * [off, off+len) of an arena; parity bytes sit at the SAME offset as the data
 * they encode (/root/reference/memcached.c:7704-7717), offsets are 16-B aligned
 * (/root/reference/ecalloc.c:176) and recovery works on 4 KiB units
 * (/root/reference/const.h:26).  Unaligned offsets and lengths are accepted
 * (slower byte path for the affected tiles), bit-exact either way.
 *
 * LIFETIME RULE (every object: plan, drainer, recovery session, recovery pool):
 * destroy the object BEFORE any stream it was used on.  An object records the streams
 * its calls used and its destroy synchronises exactly those (never the whole device);
 * a handle of a destroyed stream cannot be synchronised (it crashes the HIP runtime).
 * This is a change from the first release, whose destroy waited for the whole device.
 * The recorded list grows with every distinct stream an object is used on.  A long-lived
 * object used on short-lived streams (one per client connection) calls its
 * *_release_stream(obj, stream) before destroying such a stream: that waits for the
 * object's work on it and drops it from the list, which then stays bounded by the
 * streams alive (and the object's destroy no longer touches the dead handle).
 *
 * THREADS: every entry point may be called from any thread.  The library's shared
 * state (caches, the engine and occupancy settings) is thread-safe, and each op reads
 * the process-wide engine once, so a concurrent cec_set_engine changes later ops only.
 * A plan is immutable once created and may be used by several threads' ops at once.
 * Drainers, recovery sessions and recovery pools carry per-object state: calls on one
 * such object must not overlap (one thread at a time, as Cocytus' single worker thread
 * per process makes them).
 *
 * Coding matrix: int[(k+m)*k], row-major, MATRIX(x,y) = matrix[x*k+y]
 * (/root/reference/memcached.h:52), as returned by
 * reed_sol_big_vandermonde_distribution_matrix(k+m, k, 8)
 * (/root/reference/memcached.c:6845).  Limits: 1 <= k <= CEC_MAX_K,
 * 1 <= m <= CEC_MAX_M, k+m <= 32 (Cocytus masks are uint32_t).
 */
#ifndef COCYTUS_EC_H
#define COCYTUS_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CEC_MAX_K 16
#define CEC_MAX_M 8
#define CEC_UNIT_SIZE 4096 /* UNITSIZE, /root/reference/const.h:26; also the kernel tile */

typedef enum cec_status {
    CEC_OK = 0,
    CEC_EINVAL = -1,      /* bad argument (k/m/lid/mask/pointer/pattern index) */
    CEC_ESINGULAR = -2,   /* decode submatrix not invertible (memcached.c:7908 asserts) */
    CEC_EHIP = -3,        /* a HIP runtime call failed; see cec_last_error() */
    CEC_ENOMEM = -4,      /* device or pinned-host allocation failed */
    CEC_EOVERLAP = -5,    /* read-modify-write op on a plan whose extents overlap */
    CEC_ENODEV = -6,      /* no usable gfx950 device: there is no CPU fallback */
    CEC_EFULL = -7        /* a recovery pool has no room for the request */
} cec_status;

/* One value of a batch.  `off` addresses the arenas (item->addr, memcached.h:441);
 * `src_off` addresses the staging buffer that carries values from / to the network
 * (c->vbuf, e->vbuf: memcached.c:3646-3655, 7727-7735); `pattern` is per-op:
 *   cec_diff_update / cec_apply_diffs /
 *   cec_set_diff                       : source data shard lid j (0..k-1)
 *   cec_decode                         : index into the op's mask array
 *   other ops (encode, residual, solve): 0.
 * An index out of range (j >= k, >= n_masks, or not 0) makes the op return
 * CEC_EINVAL before anything is launched. */
typedef struct cec_extent {
    uint64_t off;
    uint64_t src_off;
    uint32_t len;
    uint32_t pattern;
} cec_extent;

/* A device-resident batch: the extents plus the 4 KiB tile work-list the kernels
 * walk (load balance across mixed 256 B .. 1 MiB values).  Build once per batch. */
typedef struct cec_plan cec_plan;

/* GF(2^8) engine used by the kernels.  Both are bit-exact and within a few % of each
 * other.  PERM looks up three 8-entry byte tables per coefficient with v_perm_b32
 * (pure VALU, no LDS); LDS stages one 256-entry product row per coefficient,
 * exp[log x + log c] built from the log / antilog tables, in LDS (one ds_read_u8 per
 * byte).  AUTO (default) runs the LDS engine only where it led PERM by more than 2 % on
 * the median of the recorded boxes: cec_decode of values of 64 KiB and
 * more (the plan's mean extent), with one mask or many.  Every other op runs PERM:
 * encodes (any size), decodes of smaller values, the diff-update, residual, solve, set
 * diff, apply, region multiply and the recovery sessions and pool. */
typedef enum cec_engine { CEC_ENGINE_PERM = 0, CEC_ENGINE_LDS = 1, CEC_ENGINE_AUTO = 2 } cec_engine;

/* ---- runtime ---- */
const char *cec_version(void);
const char *cec_last_error(void);               /* thread-local message of the last failure */
int cec_device_check(void);                     /* CEC_OK if the current device is gfx950 */
int cec_set_engine(cec_engine e);               /* process-wide; default CEC_ENGINE_AUTO */
cec_engine cec_get_engine(void);
/* The engine (CEC_ENGINE_PERM or CEC_ENGINE_LDS) the calling thread's last op chose
 * (AUTO resolved), -1 before its first op.  Diagnostics: which kernel family ran. */
int cec_last_engine(void);
/* Occupancy of the streaming kernels: at most waves_per_cu waves of one launch per CU
 * (0 = as many as fit).  Process-wide; the initial value comes from the
 * CEC_WAVES_PER_CU environment variable.  A tuning knob: every value is bit-exact. */
int cec_set_waves_per_cu(int waves_per_cu);
int cec_get_waves_per_cu(void);

/* ---- arena layout in HBM ----
 * The kernels stream every arena at the same offset at once.  Arenas carved from one
 * allocation at a stride that is an ODD number of 4 KiB pages keep those concurrent
 * streams off the same HBM channel / bank group; even strides (and separate hipMallocs,
 * by chance) collide: measured 0.386-0.395 ms vs 0.418-0.426 ms per RS(3,2) 4 KiB
 * encode + decode step.  Use these for ecmem-style arenas. */
size_t cec_arena_stride(size_t bytes);             /* smallest odd multiple of 4 KiB >= bytes */
/* count arenas of `bytes` each in one device allocation; arenas[i] = base + i * stride.
 * *slab receives the allocation (pass it to cec_arenas_free). */
int cec_arenas_alloc(int count, size_t bytes, uint8_t **arenas, void **slab);
int cec_arenas_free(void *slab);

/* ---- plans ---- */
/* extents: HOST array of n cec_extent (n >= 0).  The tile list is built on the host
 * and copied to the device on `stream`; the plan is usable by later calls on any
 * stream ordered after it.  Overlapping [off, off+len) ranges are recorded: RMW ops
 * (cec_diff_update, cec_apply_diffs) refuse such a plan with CEC_EOVERLAP. */
int cec_plan_create(cec_plan **out, const cec_extent *extents, int n, void *stream);
/* Waits for the streams the plan was used on (its upload and launches), never for the
 * device or other streams.  LIFETIME RULE (top of this header): destroy plans (and
 * sessions, drainers, pools) before the streams they were used on.  A plan used inside
 * a captured graph must outlive the graph's replays. */
int cec_plan_destroy(cec_plan *plan);
/* Before destroying `stream`: wait for this plan's work on it and stop tracking it
 * (LIFETIME RULE above).  Not used on it: no-op.  cec_plan_tracked_streams: how many
 * streams the plan's destroy would synchronise now. */
int cec_plan_release_stream(cec_plan *plan, void *stream);
int cec_plan_tracked_streams(const cec_plan *plan);
int cec_plan_num_extents(const cec_plan *plan);
int64_t cec_plan_num_tiles(const cec_plan *plan);
uint64_t cec_plan_total_bytes(const cec_plan *plan); /* sum of extent lengths */

/* ---- ops (all async on `stream`) ---- */

/* Device form of galois_w08_region_multiply:
 * add != 0: dst[i] ^= c*src[i]; add == 0: dst[i] = c*src[i]; dst == NULL: in place. */
int cec_region_multiply(const void *src, int multby, size_t nbytes, void *dst, int add,
                        void *stream);

/* Full-stripe encode over arena extents (a5): parity[p][off..] = sum_j
 * MATRIX(k+p, j) * data[j][off..].  data: k device arena bases, parity: m. */
int cec_encode(int k, int m, const int *matrix, const uint8_t *const *data,
               uint8_t *const *parity, const cec_plan *plan, void *stream);

/* Encode one contiguous range [0, len) of every arena (no plan needed). */
int cec_encode_region(int k, int m, const int *matrix, const uint8_t *const *data,
                      uint8_t *const *parity, size_t len, void *stream);

/* Fused per-SET diff-update (a4 = a2 + M x a3): for each extent with source shard
 * j = pattern: d = staging[src_off..] ^ data[j][off..]; parity[p][off..] ^=
 * MATRIX(k+p, j) * d for every p with parity[p] != NULL (a lost parity is
 * skipped, memcached.c:2692-2694); if install, data[j][off..] = new value
 * (memcached.c:5666).  Extents must not overlap (CEC_EOVERLAP). */
int cec_diff_update(int k, int m, const int *matrix, uint8_t *const *data,
                    const uint8_t *staging, uint8_t *const *parity, int install,
                    const cec_plan *plan, void *stream);

/* Data-side diff only (memcached.c:2673-2681): diff[src_off..] = staging[src_off..]
 * ^ data[pattern][off..].  diff and staging share src_off addressing. */
int cec_set_diff(int k, const uint8_t *const *data, const uint8_t *staging, uint8_t *diff,
                 const cec_plan *plan, void *stream);

/* Parity-side deferred apply of shipped diffs (memcached.c:7762-7767, the drain
 * loops at :4231, :4322, :4350, :8068): parity[off..] ^= MATRIX(lid_self, j) *
 * diffs[src_off..] with j = pattern.  Extents must not overlap (CEC_EOVERLAP). */
int cec_apply_diffs(int k, int m, const int *matrix, int lid_self, const uint8_t *diffs,
                    uint8_t *parity, const cec_plan *plan, void *stream);

/* Recovery residual on parity lid_self (recovery.c:61-96): residual[off..] =
 * arenas[lid_self][off..] ^ sum_{data lid s in mask, s != lid_self}
 * MATRIX(lid_self, s) * arenas[s][off..].  arenas: k+m bases indexed by lid (only
 * the ones the mask names are read). */
int cec_residual(int k, int m, const int *matrix, int lid_self, uint32_t mask,
                 const uint8_t *const *arenas, uint8_t *residual, const cec_plan *plan,
                 void *stream);

/* Leader solve (memcached.c:7842-7922): with n lost data lids (not in mask) and the
 * n parities in mask, out[lost_i][off..] = sum_r inv[i][r] * residuals[par_r][off..].
 * residuals: k+m bases indexed by parity lid; out: k bases indexed by data lid. */
int cec_solve(int k, int m, const int *matrix, uint32_t mask,
              const uint8_t *const *residuals, uint8_t *const *out, const cec_plan *plan,
              void *stream);

/* Fused online recovery (residual + solve in one pass, bit-exact because GF(2^8)
 * arithmetic is exact): for each extent, mask = masks[pattern]; every data lid not
 * in the mask is rebuilt into out[lid][off..] from the k participants' arenas.
 * masks follow start_recovery (memcached.c:8136-8151): exactly k lids. */
int cec_decode(int k, int m, const int *matrix, const uint32_t *masks, int n_masks,
               const uint8_t *const *arenas, uint8_t *const *out, const cec_plan *plan,
               void *stream);

/* Mask helper identical to start_recovery (memcached.c:8136-8151).  connected:
 * k+m ints.  Returns 0 if fewer than k lids are available. */
uint32_t cec_recovery_mask(int k, int m, int leader_lid, const int *connected);

/* ---- server-side batching: the parity's deferred-commit drain ----
 * Replaces the drain loops `while (done_xid < stable_xid) process_rep_command(...)`
 * (memcached.c:4231, 4322, 4350, 8068) with one call per batch of pending diffs. */
typedef struct cec_host_update {   /* one pending rep_queue_item (rep_queue.h:28-39) */
    const void *buf;               /* e->vbuf: the shipped diff, host memory (any kind) */
    uint64_t addr;                 /* e->addr: arena offset (replayed ecalloc address) */
    uint32_t len;                  /* it->nbytes */
    uint32_t src_lid;              /* data shard lid the diff came from (0..k-1) */
} cec_host_update;

typedef struct cec_drainer cec_drainer;

/* A drainer for parity lid_self owns pinned + device staging of staging_bytes (diffs
 * larger than that are applied in several rounds) and a reusable tile list. */
int cec_drainer_create(cec_drainer **out, int k, int m, const int *matrix, int lid_self,
                       size_t staging_bytes);
int cec_drainer_destroy(cec_drainer *d);
int cec_drainer_release_stream(cec_drainer *d, void *stream);   /* LIFETIME RULE, top */

/* parity[addr..] ^= MATRIX(lid_self, src_lid) * buf for every update, as the sequential
 * loop of memcached.c:7762-7767 would leave it (XOR accumulation commutes; updates
 * whose ranges overlap are put in separate launches, never raced).  Synchronous: on
 * return every update is applied and the host buffers may be reused / acked. */
int cec_drainer_apply(cec_drainer *d, const cec_host_update *updates, int n,
                      uint8_t *parity, void *stream);

/* The checks cec_drainer_apply makes on its updates before it touches anything (src_lid
 * < k, buf non-NULL when len > 0, len <= half the staging area), on the host only: CEC_OK
 * or CEC_EINVAL.  A caller with side effects per update (the server's recovery fold) runs
 * it first, so that an update the apply would refuse is refused before any of them. */
int cec_drainer_validate(const cec_drainer *d, const cec_host_update *updates, int n);

/* Launches the last cec_drainer_apply needed (>= 1 when n > 0: overlap waves x rounds). */
int cec_drainer_last_launches(const cec_drainer *d);

/* The drainer's pinned staging area (2 x staging_bytes; *capacity receives its size).
 * A server can receive diffs straight into it (conn_nread of the "rep" payload,
 * memcached.c:7727-7735, into e->vbuf carved from this area).  When every update of a
 * cec_drainer_apply call points into it, the call skips the pack copy: one H2D of the
 * used span, then the fold.  The caller must not write the area during an apply. */
uint8_t *cec_drainer_staging(cec_drainer *d, size_t *capacity);

/* ---- galois_w08_region_multiply, batched, over host memory ----
 * The unchanged server keeps its recovery state in host memory -- one malloc'd 4 KiB
 * buffer per recovery unit (recovery.c:79), the parity arena ecmem (recovery.c:81),
 * malloc'd peer replies and diffs, calloc'd solve outputs (memcached.c:7913) -- and calls
 * galois_w08_region_multiply once per unit (recovery.c:91, 123; memcached.c:7918).  This
 * runs a whole list of such calls as one staged pass (one kernel launch per overlap wave):
 *
 *   add = 0              : dst  = multby * src
 *   add = 1, base = NULL : dst ^= multby * src      (galois_w08_region_multiply(src, multby, len, dst, 1))
 *   add = 1, base != NULL: dst  = base ^ multby * src  (the first-touch copy of recovery.c:79-82,
 *                                                      then the fold of :91, fused)
 *
 * The bytes equal the calls run one by one in job order: jobs whose dst ranges overlap are
 * applied in separate launches (in job order when one of them writes; XOR accumulation
 * commutes).  A src or base range must not overlap any job's dst (CEC_EOVERLAP; base ==
 * dst is the in-place add).  Every pointer is HOST memory (pageable, pinned or registered;
 * device-resident state uses the device ops above).  Bases inside a region registered with
 * cec_host_register (the server's ecmem) are read in place through its device alias when
 * no two destinations of a staging round overlap: one copy less.  Synchronous: on return every dst
 * holds its bytes.  Lengths and alignments are arbitrary.  Staging is per calling thread:
 * mapped pinned memory, up to 2 x 24 MiB (more for one larger overlapping cluster), kept
 * for the thread's next call; batches above 4 MiB are pipelined over double-buffered
 * rounds.  A HIP failure (CEC_EHIP) may leave some destinations written and others not. */
typedef struct cec_region_job {
    const void *src;    /* region (read) */
    void *dst;          /* r2 (written) */
    const void *base;   /* see above; NULL for the plain call */
    uint32_t len;       /* nbytes */
    int32_t multby;     /* 0..255 */
    int32_t add;        /* 0 or 1 */
} cec_region_job;

int cec_region_multiply_batch(const cec_region_job *jobs, int n, void *stream);
/* Diagnostics of the calling thread's last batch: kernel launches (overlap waves x
 * rounds), staging rounds, and host wall time in microseconds spent planning (clusters,
 * waves, patterns), packing the inputs into the staging, in the GPU pass (launch to
 * completion) and unpacking the results. */
typedef struct cec_batch_stats {
    int launches, rounds;
    float plan_us, pack_us, gpu_us, unpack_us;
    int in_place_launches; /* launches that read their bases in place (cec_host_register'd) */
} cec_batch_stats;
int cec_region_multiply_batch_stats(cec_batch_stats *out);

/* ---- online recovery over 4 KiB unit ranges ----
 * One recovery request on a participating parity (recovery_queue_item,
 * recovery.h:57-69): units [unit_begin, unit_end] (UNITSIZE = 4 KiB, const.h:26) of
 * the arenas, participants `mask` (start_recovery, memcached.c:8136-8151).  The
 * residual lives in HBM.  Peer data, diffs and the other parities' residuals may be
 * host memory (pageable or pinned: staged through a pipelined pinned uploader) or
 * device memory (used in place).  All calls are synchronous: their results (device,
 * pinned or pageable) are complete on return and the caller may reuse its buffers.
 * destroy waits only for the streams the session's calls used; work the CALLER queued
 * on cec_recovery_residual(r) (e.g. shipping it with cec_copy on another stream) must
 * be complete before destroy, since the residual's memory is then reused. */
typedef struct cec_recovery cec_recovery;

int cec_recovery_create(cec_recovery **out, int k, int m, const int *matrix, int lid_self,
                        uint32_t mask, int unit_begin, int unit_end,
                        const uint8_t *parity_arena /* device: this parity's arena */,
                        void *stream);
int cec_recovery_destroy(cec_recovery *r);
int cec_recovery_release_stream(cec_recovery *r, void *stream); /* LIFETIME RULE, top */

/* recovery_recover_units (recovery.c:61-96): data peer peer_lid (in mask, not yet
 * applied) sent its raw bytes of the whole range (nbuf bytes).  The first peer also
 * copies the parity units in (first touch, recovery.c:79-82), fused into one pass. */
int cec_recovery_add_peer(cec_recovery *r, int peer_lid, const void *units, void *stream);

/* recovery_try_update_unit (recovery.c:99-131): a diff of len bytes at arena address
 * addr from data peer peer_lid reached this parity during recovery.  It is folded into
 * the residual where the range is touched and the peer has not contributed yet.
 * Returns the number of units folded (>= 0) or a negative cec_status. */
int cec_recovery_fold_update(cec_recovery *r, int peer_lid, uint64_t addr, const void *diff,
                             uint32_t len, void *stream);

/* check_recovery_1st_completeness (memcached.c:2522-2545): 1 when every data lid of
 * the mask has contributed, else 0. */
int cec_recovery_complete(const cec_recovery *r);

/* The residual (device memory, cec_recovery_bytes(r) bytes). */
const uint8_t *cec_recovery_residual(const cec_recovery *r);
uint64_t cec_recovery_bytes(const cec_recovery *r);

/* Leader (complete_recovery_bottom_half, memcached.c:7842-7922): C[j] = residual of
 * the j-th parity in the mask (this session's own for lid_self; peer_residuals[lid]
 * for the others, host or device); out[lost lid] (host or device, nbuf bytes each) =
 * sum_j inv[i][j] * C[j] for the n lost data lids. */
int cec_recovery_solve(cec_recovery *leader, const void *const *peer_residuals,
                       void *const *out, void *stream);

/* The last data peer and the leader solve (= cec_recovery_add_peer of that peer, then
 * cec_recovery_solve; same bytes, same residual afterwards).  With device or pinned
 * buffers it is ONE pass: the kernel reads the peer's bytes and writes the rebuilt
 * bytes (over PCIe in both directions at once for pinned host memory).  Pageable
 * buffers take the two-step path.  EINVAL if peer is not the last data peer. */
int cec_recovery_finish(cec_recovery *leader, int peer_lid, const void *units,
                        const void *const *peer_residuals, void *const *out, void *stream);

/* ---- background recovery of many small unit ranges ----
 * The idle recoverer issues one 4 KiB unit per request, up to TOO_MANY_RECOVERY = 85
 * in flight (idle_event_handler, memcached.c:5712-5734; const.h:27).  A pool keeps
 * every in-flight request's residual in one HBM buffer: replies are queued with a
 * host memcpy into per-peer pinned staging, and cec_recovery_pool_flush folds all of
 * them in ONE launch (first-touch parity copy fused, recovery.c:61-96).  The leader
 * solves any number of complete single-loss requests in one launch into the lost
 * lids' arenas (memcached.c:7842-7922).  Same bytes as the reference chain. */
typedef struct cec_recovery_pool cec_recovery_pool;

int cec_recovery_pool_create(cec_recovery_pool **out, int k, int m, const int *matrix, int lid_self,
                             const uint8_t *parity_arena /* device */, int capacity_units);
int cec_recovery_pool_destroy(cec_recovery_pool *pool);
int cec_recovery_pool_release_stream(cec_recovery_pool *pool, void *stream); /* LIFETIME RULE */
/* start_recovery / do_recovery: returns the request id (>= 0), CEC_EFULL when the pool
 * has no unit_end - unit_begin + 1 free contiguous units, or CEC_EINVAL. */
int cec_recovery_pool_begin(cec_recovery_pool *pool, uint32_t mask, int unit_begin, int unit_end);
/* complete_recovery_nread: data peer peer_lid's raw units of request id (host or
 * device).  Queued, not yet folded. */
int cec_recovery_pool_add_peer(cec_recovery_pool *pool, int id, int peer_lid, const void *units);
/* The same for n replies of an event-loop pass (reply i: request ids[i], data peer
 * peer_lids[i], bytes units[i]), in one call: every reply is checked as add_peer checks it
 * (and no (request, peer) pair twice) before any is queued; CEC_EINVAL queues nothing. */
int cec_recovery_pool_add_peers(cec_recovery_pool *pool, const int *ids, const int *peer_lids,
                                const void *const *units, int n);
/* Where peer peer_lid's reply for request id may be received in place (pinned, mapped;
 * *len bytes): add_peer on this pointer copies nothing. */
uint8_t *cec_recovery_pool_staging(cec_recovery_pool *pool, int id, int peer_lid, size_t *len);
/* Fold every queued reply in one launch; returns the requests folded (>= 0). */
int cec_recovery_pool_flush(cec_recovery_pool *pool, void *stream);
/* The same launch also solves every request it completes that is a single loss led by
 * this parity: out[lost lid] (k device arenas by data lid, arena-addressed) =
 * inv * residual.  Returns the requests solved; cec_recovery_pool_solved tells which. */
int cec_recovery_pool_flush_solve(cec_recovery_pool *pool, uint8_t *const *out, void *stream);
/* 1 while the request's rebuilt bytes are current: a solve (fused or explicit) wrote them
 * and no fold_update has changed its residual since (a lost lid's diff, recovery.c:116-120,
 * clears it). */
int cec_recovery_pool_solved(const cec_recovery_pool *pool, int id);
/* check_recovery_1st_completeness: every data lid of the request's mask applied or queued. */
int cec_recovery_pool_complete(const cec_recovery_pool *pool, int id);
/* recovery_try_update_unit for every request of the pool (flushes first); returns the
 * units folded (>= 0) or a negative cec_status. */
int cec_recovery_pool_fold_update(cec_recovery_pool *pool, int peer_lid, uint64_t addr, const void *diff,
                                  uint32_t len, void *stream);
/* The same for a drain window: every update u[i] (host buffers; any data lid) folded as
 * cec_recovery_pool_fold_update would fold it, in one upload and one launch per overlap
 * wave (flushes first).  units[i] (optional) = update i's units folded; returns their sum. */
int cec_recovery_pool_fold_updates(cec_recovery_pool *pool, const cec_host_update *u, int n, int *units,
                                   void *stream);
/* Leader, single loss: out[lost lid] (k device arenas by data lid, arena-addressed) =
 * inv * residual for every listed complete request, one launch (flushes first). */
int cec_recovery_pool_solve(cec_recovery_pool *pool, const int *ids, int n, uint8_t *const *out,
                            void *stream);
/* For a server whose recovery state stays in host memory (integration/
 * cocytus_recovery_pool.c): the same two solves, but into the pool's own mapped pinned
 * output at each request's slots instead of an arena, so no unit the caller has not
 * chosen is written (fill_completed_recovered_data skips sub_flags == 2 units,
 * memcached.c:7967-8000).  The bytes are fenced for the host when the call returns. */
int cec_recovery_pool_flush_solve_host(cec_recovery_pool *pool, void *stream);
int cec_recovery_pool_solve_host(cec_recovery_pool *pool, const int *ids, int n, void *stream);
/* Request id's rebuilt bytes (*len = its units x 4 KiB) after a _host solve, while
 * cec_recovery_pool_solved(id) holds; NULL otherwise.  Valid until the request ends. */
const uint8_t *cec_recovery_pool_output(const cec_recovery_pool *pool, int id, size_t *len);
/* Non-leader: copy request id's residual (its units x 4 KiB) to dst (host or device). */
int cec_recovery_pool_residual(cec_recovery_pool *pool, int id, void *dst, void *stream);
/* recovery_req_remove: release the request's units. */
int cec_recovery_pool_end(cec_recovery_pool *pool, int id);
int cec_recovery_pool_active(const cec_recovery_pool *pool);

/* ---- process-wide caches ----
 * Coefficient tables are uploaded once per distinct content (asynchronously, on the
 * caller's stream; another stream waits on the upload event) and kept in an LRU cache
 * of at most pattern_entry_limit sets per device.  Evicting synchronises the device once
 * per batch of victims; a fixed set of codes and masks never evicts.  Tables used inside
 * a stream capture stay for the life of the process (the graph holds their address).
 * Idle device and pinned buffers of plans, recovery sessions, drainers, pools and the
 * drop-in are kept for reuse (freeing them would wait for the whole device), capped at
 * 2 GiB device / 1 GiB pinned / 512 MiB mapped pinned.  At process exit the library
 * synchronises each device it cached state for and frees it. */
typedef struct cec_cache_info {
    uint64_t pattern_entries;      /* coefficient-table sets cached on this device */
    uint64_t pattern_bytes;        /* their device bytes (a pinned mirror each as well) */
    uint64_t pattern_uploads;      /* sets uploaded since start (misses) */
    uint64_t pattern_evictions;    /* LRU evictions since start */
    uint64_t pattern_entry_limit;
    uint64_t device_cached_bytes;  /* idle device buffers held for reuse (all devices) */
    uint64_t pinned_cached_bytes;  /* idle pinned host buffers held for reuse */
} cec_cache_info;
int cec_cache_get_info(cec_cache_info *out);       /* current device */
int cec_cache_set_pattern_limit(int entries);      /* default 4096 (CEC_PATTERN_CACHE_ENTRIES) */
/* Free every idle cached buffer and every coefficient-table set not used by a captured
 * graph (synchronises the current device first). */
int cec_cache_trim(void);

/* ---- completion record (diagnostics) ----
 * How the calling thread's last synchronous completion (the drop-in
 * galois_w08_region_multiply, cec_recovery_fold_update / _solve / _finish,
 * cec_recovery_pool_flush / _flush_solve / _fold_update / _solve) made its results
 * visible to the host on return.  A result in
 * host-visible memory (pinned, mapped or managed) may still sit in the L2 of the XCD
 * that wrote it; it is visible only if every writing wave ended with a system-scope
 * release or a system-scope fence ran behind the op.  Tests assert the protocol with it
 * on any box, whether or not the box's host mappings expose a missing release. */
typedef struct cec_sync_record {
    uint64_t seq;           /* synchronous completions on this thread so far */
    int host_results;       /* the op wrote host-visible memory */
    int waves_released;     /* every writing wave ended with a system-scope release */
    int fenced;             /* a system-scope fence ran behind the op (fence event or stream sync) */
} cec_sync_record;
int cec_last_sync(cec_sync_record *out);

/* ---- test hooks (host only, launch nothing themselves; not for servers) ----
 * cec_internal_check_launch_layout: the launch-time check every op's launch runs, on one
 * pattern reading in_slots and writing out_slots, against the kernel argument block built
 * from bases[0..n_bases) -- the two-slot block of the narrow 1 x 1 kernels (narrow != 0)
 * or the full one.  CEC_OK, or CEC_EINVAL where the launch would be refused (a slot the
 * block does not carry, or a NULL base).
 * cec_internal_store_policy: the store policy parsed from CEC_STORE_POLICY (0 auto,
 * 1 non-temporal, 2 write-through; unknown values warn once and mean auto) and, in
 * *wt_max_bytes, auto's write-through limit (CEC_WT_MAX_BYTES, default 512 MiB). */
int cec_internal_check_launch_layout(int narrow, const int *in_slots, int n_in, const int *out_slots,
                                     int n_out, const void *const *bases, int n_bases);
int cec_internal_store_policy(uint64_t *wt_max_bytes);
/* cec_internal_fail_launch: fault injection for the error paths (tests only) -- the calling
 * thread's next `after` kernel launches run and the one after them fails as a HIP error
 * would (CEC_EHIP, nothing launched); then the hook disarms.  after < 0 disarms it. */
int cec_internal_fail_launch(int after);

/* ---- stream / event helpers, so C and ctypes callers need no HIP header ----
 * Events are for timing: recorded without the system-scope fence, so waiting on one
 * does not make results written into host memory visible.  Use cec_stream_synchronize
 * (or a synchronous call) before reading those. */
int cec_event_create(void **ev);
int cec_event_destroy(void *ev);
int cec_event_record(void *ev, void *stream);
int cec_event_elapsed_ms(void *start, void *stop, float *ms); /* synchronises on stop */
int cec_stream_synchronize(void *stream);
/* Device selection for C callers (one host thread per GPU): the calling
 * thread's current device, as hipGetDeviceCount / hipSetDevice. */
int cec_device_count(int *count);
int cec_set_device(int device);
/* A non-blocking stream of the current device (each is a hardware queue: use one per
 * thread). */
int cec_stream_create(void **stream);
int cec_stream_destroy(void *stream);
/* Async copy between any host / device buffers (arena bytes to and from the server's
 * buffers); complete after cec_stream_synchronize(stream). */
int cec_copy(void *dst, const void *src, size_t n, void *stream);
/* A host arena the server keeps in its own memory (ecmem: mmap'd, ecmem.h:36-42) made
 * reachable by the kernels: page-locked and mapped once
 * (hipHostRegister), *device_alias = its address for the device ops (cec_encode,
 * cec_drainer_apply, ...; results are complete for the host after the op's stream
 * synchronises, or on return of the synchronous calls).  Unregister before freeing it. */
int cec_host_register(void *p, size_t bytes, uint8_t **device_alias);
int cec_host_unregister(void *p);

#ifdef __cplusplus
}
#endif
#endif /* COCYTUS_EC_H */
