/*
 * integration/cocytus_recovery_pool.h -- server-side glue, second placement: the parity's
 * online recovery coalesced onto a cec_recovery_pool (INTEGRATION.md
 * §3.3).  Same role as cocytus_recovery.{h,c}, same server types (the reference's
 * recovery.h, used where it lies), same flag logic and return values; what differs is where
 * the units' bytes live:
 *
 *   cocytus_recovery.c        unit->data, malloc'd host buffers, as the unchanged server;
 *                             every fold and solve is a cec_region_multiply_batch over host
 *                             memory (staged through pinned buffers, PCIe both ways).
 *   cocytus_recovery_pool.c   the pool's residual in HBM: a reply is a host memcpy into the
 *                             pool's mapped staging (or is received there in place), and one
 *                             launch per event-loop pass folds every queued reply (first-touch
 *                             parity copy fused) and solves every request it completes into
 *                             the pool's mapped output, which the server reads in place.
 *                             unit->data stays NULL: the flags are kept as the reference keeps
 *                             them, the bytes are the pool's.
 *
 * The server lines that read unit->data change with the placement: send_recovered_data
 * (memcached.c:7823-7839) sends cocytus_rpool_residual's bytes, the leader's bottom half
 * (memcached.c:7842-7962) takes cocytus_rpool_data's; recovery_req_remove (recovery.c:
 * 190-211) and restart_failed_recovery's reset (memcached.c:8019-8046) call cocytus_rpool_end
 * for the request first.  The parity arena is the device view of ecmem: a device arena, or
 * the alias cec_host_register returns for the unchanged server's host ecmem (the first-touch
 * copy then reads it over PCIe, in the same launch).
 *
 * Timing: the bottom half runs at cocytus_rpool_flush, over the residual as it is then (as
 * cocytus_recovery_solve_defer): call the flush once per event-loop pass, after the pass's
 * replies and drains, and act on the solved requests after it.
 *
 * Errors: a negative cec_status; the reference's assert()s are refused before anything
 * changes (CEC_EINVAL), as in cocytus_recovery.c.  A failed GPU pass leaves the recovery
 * state undefined: the process must stop.
 */
#ifndef COCYTUS_RECOVERY_POOL_H
#define COCYTUS_RECOVERY_POOL_H

#include <stdint.h>

#include <cocytus_ec.h>

#include "recovery.h" /* the server's: struct recovery, recovery_unit, recovery_queue_item */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cocytus_rpool cocytus_rpool;

/* One per parity process, called from the thread that runs its recovery (like struct
 * recovery itself, it takes no locks).  parity_dev: this parity's arena as the device sees
 * it (above); queue_cap: recovery.queue.cap (requests are keyed by their slot in
 * recovery.queue.items);
 * capacity_units: residual slots (at least the largest request's units; the idle recoverer
 * needs 85).  stream: the worker thread's (NULL: the default stream). */
int cocytus_rpool_create(cocytus_rpool **out, int k, int m, const int *matrix, int self_lid, const void *parity_dev,
                         int queue_cap, int capacity_units, void *stream);
/* Pending work is dropped; every request's buffers are freed. */
void cocytus_rpool_destroy(cocytus_rpool *g);

/* After recovery_req_add (do_recovery / the recover_units handler): the request's residual
 * slots.  CEC_EFULL when the pool has no room (back off, as TOO_MANY_RECOVERY does). */
int cocytus_rpool_begin(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit);
/* Before recovery_req_remove, and for each request restart_failed_recovery resets: the
 * slots and any rebuilt bytes are released.  A request with none is a no-op (an aborted
 * request is removed later, memcached.c:2602-2606). */
int cocytus_rpool_end(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit);

/* recovery_recover_units (recovery.c:61-96) for rqit's reply from data peer peerid (its
 * units x UNITSIZE bytes at data): the reference's checks and flags now (first touch: UPDATE
 * and settings.lid; then the peer), the fold queued in the pool.  data is copied unless it
 * is cocytus_rpool_staging's buffer; the caller keeps it. */
int cocytus_rpool_recover_units(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit,
                                int peerid, const char *data);
/* Where peer peerid's reply for rqit may be received in place (c->ritem): pinned and
 * device-mapped, the request's units x UNITSIZE bytes.  NULL if rqit has no slots. */
char *cocytus_rpool_staging(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit, int peerid);

/* recovery_try_update_unit (recovery.c:99-131): the return value and touch_flags as the
 * reference; the units it would fold are folded in the pool now (one launch when any).
 * CEC_EINVAL if the pool's state disagrees with the flags (a reset without
 * cocytus_rpool_end). */
int cocytus_rpool_try_update_unit(cocytus_rpool *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                                  int peerid, uint64_t addr, const char *data, uint32_t size);
/* The same over a drain window (need[i] per update, in xid order): every fold of the window
 * in one cec_recovery_pool_fold_updates. */
int cocytus_rpool_try_update_units(cocytus_rpool *g, struct recovery *r, char *const *touch_flags,
                                   const char *sub_flags, const cec_host_update *u, int n, int *need);

/* send_recovered_data's bytes (a non-leader): rqit's residual, units x UNITSIZE, into buf.
 * Folds what is queued first. */
int cocytus_rpool_residual(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit, char *buf);

/* complete_recovery_bottom_half (memcached.c:7842-7922), queued for the next flush: *n_out
 * = the lost data lids.  C = this parity's residual (if in the mask) and
 * rqit->data_from_parity for the other parities of the mask (keep them until the flush).
 * A single loss led by this parity is solved in the flush's own launch; any other mask
 * through one cec_region_multiply_batch after it. */
int cocytus_rpool_solve(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit, int *n_out);
/* Fold every queued reply and run every queued solve.  Returns the solves run (>= 0). */
int cocytus_rpool_flush(cocytus_rpool *g);
/* After the flush that ran rqit's solve: data[x] of the bottom half (the x-th lost data lid,
 * units x UNITSIZE bytes), for fill_completed_recovered_data or the scatter send
 * (memcached.c:7935-7962).  Valid until cocytus_rpool_end; NULL before the solve ran, and
 * for a single loss solved in the pool also once a later fold has changed its residual (a
 * lost lid's SET: read the bytes right after the flush, as the bottom half does). */
const char *cocytus_rpool_data(const cocytus_rpool *g, const struct recovery *r, const struct recovery_queue_item *rqit,
                               int x);
/* Queued solves not yet run. */
int cocytus_rpool_pending(const cocytus_rpool *g);

/* The drain glue's batched fold hook (cocytus_drain_hooks.try_update_batch). */
typedef struct cocytus_rpool_fold_ctx {
    cocytus_rpool *g;
    struct recovery *r;
    char *touch_flags[32]; /* peers[lid].touch_flags by lid */
    const char *sub_flags;
} cocytus_rpool_fold_ctx;
int cocytus_rpool_fold_hook(const cec_host_update *u, int n, int *need, void *ctx);

#ifdef __cplusplus
}
#endif
#endif /* COCYTUS_RECOVERY_POOL_H */
