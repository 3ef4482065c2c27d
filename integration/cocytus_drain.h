/*
 * integration/cocytus_drain.h -- server-side glue: the parity process's deferred-commit
 * drain loops batched onto libcocytus_ec.
 *
 * This file and cocytus_drain.c belong in the Cocytus server tree (add cocytus_drain.c to
 * memcached_SOURCES next to rep_queue.c); they are not part of libcocytus_ec.so.  They
 * use the server's own queue types (rep_queue.h) unchanged.
 *
 * The loops they replace run, on a parity process, every queued SET diff of data peer
 * `lid` up to the stable xid the peer announced:
 *     while (peers[lid].done_xid < got_stable_xid)
 *         process_rep_command(c, ++peers[lid].done_xid, -1);
 * (/root/reference/memcached.c:4231, 4322, 4350; process_queued_items, :8068).  Per xid,
 * process_rep_command (:7739-7798) finds the item (rep_queue_find), folds the diff into an
 * in-progress recovery (recovery_try_update_unit, recovery.c:99-131) and, if that says the
 * parity must take it, multiplies it into the parity arena:
 *     galois_w08_region_multiply(e->vbuf, MATRIX(settings.lid, lid), it->nbytes,
 *                                ecmem_get(&ecmem, addr), 1);
 * then stores the item in the peer's hash table and marks the entry done.
 *
 * cocytus_drain_gf() does the GF half of the whole loop in one batch: it collects every
 * entry with done_xid < xid <= stable_xid in xid order, asks the recovery hook about each
 * (in that order, as the loop would), and applies all the diffs the hook lets through with
 * ONE cec_drainer_apply (one H2D + one fold launch; overlapping diffs are put in separate
 * waves, XOR accumulation commutes, so the parity bytes equal the sequential loop's).  The
 * server then runs the rest of process_rep_command per xid, without its two GF lines.
 */
#ifndef COCYTUS_DRAIN_H
#define COCYTUS_DRAIN_H

#include <stdint.h>

#include <cocytus_ec.h>

#ifdef __cplusplus
extern "C" {
#endif

struct rep_queue; /* rep_queue.h (the server's) */

typedef struct cocytus_drain_hooks {
    /* it->nbytes of the queued item (items.h); the entry's vnbytes is its buffer's
     * capacity, which may exceed the value (memcached.c:7727-7731). */
    uint32_t (*item_nbytes)(void *item, void *ctx);
    /* recovery_try_update_unit(&recovery, lid, addr, buf, nbytes) (recovery.c:99-131):
     * nonzero = the parity arena takes the diff.  NULL: no recovery state, every diff is
     * applied. */
    int (*try_update)(int lid, uint64_t addr, char *buf, uint32_t nbytes, void *ctx);
    void *ctx;
    /* The same fold for the whole window at once (cocytus_recovery.h: cocytus_fold_hook,
     * one batch for every unit piece of every update): need[i] = try_update's answer for
     * u[i]; returns >= 0, or a negative cec_status.  Used instead of try_update when set. */
    int (*try_update_batch)(const cec_host_update *u, int n, int *need, void *ctx);
} cocytus_drain_hooks;

/* The entries of q with done_xid < xid <= stable_xid, in xid order, as cec_host_updates
 * {e->vbuf, e->addr, item_nbytes(e->item), lid} in out[0..n).  Returns n, or
 *   CEC_EINVAL  an xid of the range is not queued (process_rep_command asserts), or bad args;
 *   CEC_EFULL   more than cap entries (drain in several calls: raise done_xid by cap).
 * Host only: reads the queue, touches no device. */
int cocytus_drain_collect(const struct rep_queue *q, int lid, uint64_t done_xid, uint64_t stable_xid,
                          const cocytus_drain_hooks *hooks, cec_host_update *out, int cap);

/* The GF half of the drain loop above, batched: collect, check every entry as
 * cec_drainer_apply will (cec_drainer_validate: nothing is folded for a window the apply
 * would refuse), ask the recovery fold about each entry in xid order (hooks->try_update,
 * or hooks->try_update_batch once), then ONE cec_drainer_apply of the diffs it let through
 * into the parity arena (device or registered host memory; synchronous, like the loop).
 * `scratch`: cap cec_host_updates.  Returns the number of diffs applied (>= 0) or a
 * negative cec_status.  A failure after the folds ran (the apply's HIP error) leaves the
 * recovery units ahead of the arena: the recovery state is inconsistent and the process
 * must stop (retrying the window would fold its diffs twice).  The caller then runs, per
 * xid, the rest of process_rep_command (store the item, mark done, flush). */
int cocytus_drain_gf(const struct rep_queue *q, int lid, uint64_t done_xid, uint64_t stable_xid,
                     const cocytus_drain_hooks *hooks, cec_drainer *drainer, uint8_t *parity,
                     void *stream, cec_host_update *scratch, int cap);

#ifdef __cplusplus
}
#endif
#endif /* COCYTUS_DRAIN_H */
