/*
 * integration/cocytus_recovery.h -- server-side glue: the parity process's online-recovery
 * arithmetic batched onto libcocytus_ec.
 *
 * Like cocytus_drain.{h,c}, this file and cocytus_recovery.c belong in the Cocytus server
 * tree (add cocytus_recovery.c to memcached_SOURCES next to recovery.c); they are not part
 * of libcocytus_ec.so.  They include the server's own recovery.h and work on its types
 * unchanged: struct recovery (the per-unit flags and the malloc'd 4 KiB unit buffers),
 * struct recovery_queue_item (mask, unit range, data_from_parity) and struct ecmem.  The
 * recovery state stays where the unchanged server keeps it -- host memory -- so the rest
 * of recovery.c and memcached.c (check_recovery_1st_completeness, send_recovered_data,
 * recovery_req_remove, restart_failed_recovery, fill_completed_recovered_data) run as they
 * are, on the same flags and the same bytes.
 *
 * What changes is the arithmetic.  The reference calls galois_w08_region_multiply once per
 * 4 KiB unit:
 *     recovery_recover_units      recovery.c:61-96     one call per unit of the range
 *     recovery_try_update_unit    recovery.c:99-131    one call per unit a SET touches
 *     complete_recovery_bottom_half memcached.c:7842-7922  n x n calls over nbuf
 * and each call through the drop-in is a synchronous GPU round trip (11-13 us for 4 KiB).
 * Here each of those loops is ONE cec_region_multiply_batch (one staged pass, one kernel
 * launch per overlap wave), with the flag logic of the reference applied on the host, in
 * the reference's order, before any byte changes.
 *
 * The idle recoverer (idle_event_handler, memcached.c:5712-5734) keeps up to
 * TOO_MANY_RECOVERY = 85 single-unit requests in flight (const.h:27).  The *_defer calls
 * let the server queue every reply (and every leader solve) of an event-loop pass and run
 * them with cocytus_recovery_flush: one batch for all the folds, one for all the solves.
 *
 * Errors: a negative cec_status.  The checks the reference makes with assert() (a unit
 * already recovered, a peer applied twice, a first touch of a unit that holds data, a
 * singular submatrix) are made before anything changes and return CEC_EINVAL /
 * CEC_ESINGULAR.  A failure of the GPU pass itself (CEC_EHIP) leaves the units' bytes
 * undefined: the recovery cannot continue and the process must stop, as it would on the
 * reference's assert.
 */
#ifndef COCYTUS_RECOVERY_H
#define COCYTUS_RECOVERY_H

#include <stdint.h>

#include <cocytus_ec.h>

#include "recovery.h" /* the server's: struct recovery, recovery_unit, recovery_queue_item, ecmem */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cocytus_rglue cocytus_rglue;

/* One per parity process: code (k, m, MATRIX as reed_sol_big_vandermonde_distribution_matrix
 * returned it, memcached.c:6845), settings.lid of this parity, the stream of the worker
 * thread (NULL: the default stream). */
int cocytus_rglue_create(cocytus_rglue **out, int k, int m, const int *matrix, int self_lid, void *stream);
/* Flushes nothing: pending deferred work is dropped (owned reply buffers are freed). */
void cocytus_rglue_destroy(cocytus_rglue *g);

/* recovery_recover_units (recovery.c:61-96) for the whole unit range [ubegin, uend] in one
 * batch: data peer `peerid`'s raw units (nbuf = (uend-ubegin+1)*UNITSIZE bytes at data).
 * Per unit, as the reference: not recovered, peer not yet applied (else CEC_EINVAL, nothing
 * changed); first touch: unit->data = malloc(UNITSIZE) holding the parity unit
 * (ecmem_get(ecm, i*UNITSIZE)), UPDATE and settings.lid flags set; peer flag set; unit->data
 * ^= MATRIX(self, peerid) * unit of data.  The first-touch copy is fused into the fold. */
int cocytus_recover_units_gf(cocytus_rglue *g, struct recovery *r, struct ecmem *ecm, int peerid, int ubegin,
                             int uend, const char *data);

/* recovery_try_update_unit (recovery.c:99-131) for one SET diff of `size` bytes at arena
 * address addr from data lid peerid, its unit pieces in one batch.  Returns what the
 * reference returns (the pieces whose unit is not sub_flags == 2: the parity must take the
 * diff if > 0) and, like it, sets touch_flags[unit] = 1 for every unit touched
 * (peers[peerid].touch_flags).  sub_flags may be NULL (no substitute recovery running). */
int cocytus_try_update_unit_gf(cocytus_rglue *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                               int peerid, uint64_t addr, const char *data, uint32_t size);

/* The same for a whole drain window (the updates cocytus_drain_collect returns, in xid
 * order, each from data lid u[i].src_lid): need[i] = recovery_try_update_unit's return for
 * u[i]; every fold of every update in ONE batch.  touch_flags[lid] = peers[lid].touch_flags.
 * The folds only write recovery units and the parity apply only the arena, so folding the
 * window before applying it leaves the bytes of both as the per-xid loop would. */
int cocytus_try_update_units_gf(cocytus_rglue *g, struct recovery *r, char *const *touch_flags,
                                const char *sub_flags, const cec_host_update *u, int n, int *need);

/* complete_recovery_bottom_half's arithmetic (memcached.c:7842-7922): C = this parity's
 * units of the request (if it is in the mask) and rqit->data_from_parity[lid] for the other
 * parities of the mask, ascending lid; tmpmat = MATRIX rows of those parities at the lost
 * data columns; inv = jerasure_invert_matrix(tmpmat); data[i] = sum_j inv[i][j] * C[j].
 * On return *n_out = n (lost data lids) and data[0..n) are malloc'd nbuf-byte buffers (the
 * reference's calloc'd data[]), ready for fill_completed_recovered_data / the scatter sends
 * (memcached.c:7935-7962).  Nothing of the request is freed (the server's lines that free C
 * and data_from_parity stay).  data must hold room for m pointers. */
int cocytus_recovery_solve_gf(cocytus_rglue *g, struct recovery *r, const struct recovery_queue_item *rqit,
                              char **data, int *n_out);

/* ---- coalescing (the idle recoverer: many single-unit requests per event-loop pass) ---- */

/* cocytus_recover_units_gf, deferred: the flags and first-touch copies are made now, as the
 * reference makes them when the reply arrives (so completeness checks and
 * recovery_try_update_unit's skip rules see the reference's state); the fold is queued for
 * cocytus_recovery_flush.  take != 0: the glue frees `data` after the flush (the server
 * detaches c->vbuf, as complete_recovery_gather_nread does).  Until the flush, the request's
 * unit bytes are not final: flush before send_recovered_data, the bottom half or
 * recovery_req_remove of the request.  Folds of later SET diffs (cocytus_try_update_*_gf)
 * may run before the flush: they XOR into the same units and XOR accumulation commutes. */
int cocytus_recover_units_defer(cocytus_rglue *g, struct recovery *r, struct ecmem *ecm, int peerid, int ubegin,
                                int uend, char *data, int take);

/* cocytus_try_update_unit_gf / _units_gf, deferred: the return values and touch_flags
 * now, the folds queued for cocytus_recovery_flush (same rule: flush before the units'
 * bytes are read).  The pieces to fold are copied (the diff buffers are freed by
 * rep_queue_flush as soon as the xid is processed). */
int cocytus_try_update_unit_defer(cocytus_rglue *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                                  int peerid, uint64_t addr, const char *data, uint32_t size);
int cocytus_try_update_units_defer(cocytus_rglue *g, struct recovery *r, char *const *touch_flags,
                                   const char *sub_flags, const cec_host_update *u, int n, int *need);

/* cocytus_recovery_solve_gf, deferred: data[0..*n_out) are allocated now and filled by the
 * next cocytus_recovery_flush (after that flush's folds). */
int cocytus_recovery_solve_defer(cocytus_rglue *g, struct recovery *r, const struct recovery_queue_item *rqit,
                                 char **data, int *n_out);

/* Run every queued fold (one batch), then every queued solve (one batch).  Returns the
 * number of queued requests run (folds + solves) or a negative cec_status.  On a failure
 * the queues are kept but some folds may have landed: the recovery state is undefined and
 * the process must stop (a retry could fold twice); the data[] buffers of queued solves
 * stay the caller's to free. */
int cocytus_recovery_flush(cocytus_rglue *g);

/* Queued requests (folds + solves) not yet flushed. */
int cocytus_recovery_pending(const cocytus_rglue *g);
/* The queued jobs themselves (diagnostics and tests: what the next flush will run). */
int cocytus_recovery_queued(const cocytus_rglue *g, const cec_region_job **folds, int *n_folds,
                            const cec_region_job **solves, int *n_solves);

/* The drain glue's batched fold hook (cocytus_drain_hooks.try_update_batch): ctx is a
 * cocytus_fold_ctx. */
typedef struct cocytus_fold_ctx {
    cocytus_rglue *g;
    struct recovery *r;
    char *touch_flags[32]; /* peers[lid].touch_flags by lid */
    const char *sub_flags;
    int defer; /* queue the folds for cocytus_recovery_flush instead of running them */
} cocytus_fold_ctx;
int cocytus_fold_hook(const cec_host_update *u, int n, int *need, void *ctx);

#ifdef __cplusplus
}
#endif
#endif /* COCYTUS_RECOVERY_H */
