/*
 * integration/cocytus_drain.c -- the parity drain loops batched onto libcocytus_ec
 * (see cocytus_drain.h).  Server-side glue: compiled in the Cocytus tree against its own
 * rep_queue.h (the queue ring: entries [tail, head), index i at items[i % cap],
 * /root/reference/rep_queue.h:28-47, rep_queue.c:30-80).
 */
#include "cocytus_drain.h"

#include <stdlib.h>
#include <string.h>

#include "rep_queue.h"

int cocytus_drain_collect(const struct rep_queue *q, int lid, uint64_t done_xid, uint64_t stable_xid,
                          const cocytus_drain_hooks *hooks, cec_host_update *out, int cap)
{
    if (!q || !hooks || !hooks->item_nbytes || lid < 0 || cap < 0 || (cap && !out)) return CEC_EINVAL;
    if (stable_xid <= done_xid) return 0;
    if (stable_xid - done_xid > (uint64_t)cap) return CEC_EFULL;
    const int n = (int)(stable_xid - done_xid);
    if (q->cap == 0 || !q->items || q->head - q->tail > q->cap) return CEC_EINVAL; /* not a queue */
    char *seen = calloc((size_t)n, 1);
    if (!seen) return CEC_ENOMEM;
    /* rep_queue_find's walk: tail .. head in ring order; the first entry of an xid wins */
    for (uint32_t i = q->tail; i != q->head; ++i) {
        const struct rep_queue_item *e = &q->items[i % q->cap];
        if (e->xid <= done_xid || e->xid > stable_xid) continue;
        const int slot = (int)(e->xid - done_xid - 1);
        if (seen[slot]) continue;
        seen[slot] = 1;
        out[slot].buf = e->vbuf;
        out[slot].addr = e->addr;
        out[slot].len = hooks->item_nbytes(e->item, hooks->ctx);
        out[slot].src_lid = (uint32_t)lid;
    }
    int missing = 0;
    for (int s = 0; s < n; ++s) missing |= !seen[s];
    free(seen);
    return missing ? CEC_EINVAL : n;
}

int cocytus_drain_gf(const struct rep_queue *q, int lid, uint64_t done_xid, uint64_t stable_xid,
                     const cocytus_drain_hooks *hooks, cec_drainer *drainer, uint8_t *parity,
                     void *stream, cec_host_update *scratch, int cap)
{
    if (!drainer || !parity) return CEC_EINVAL;
    const int n = cocytus_drain_collect(q, lid, done_xid, stable_xid, hooks, scratch, cap);
    if (n <= 0) return n;
    /* the folds below have side effects: refuse a window the apply would refuse first */
    int rc = cec_drainer_validate(drainer, scratch, n);
    if (rc) return rc;
    /* process_rep_command's order: the recovery fold decides, per xid, whether the
     * parity arena takes the diff (memcached.c:7758-7767) */
    int m = 0;
    if (hooks->try_update_batch) {
        int *need = malloc(sizeof(int) * (size_t)n);
        if (!need) return CEC_ENOMEM;
        rc = hooks->try_update_batch(scratch, n, need, hooks->ctx);
        if (rc < 0) {
            free(need);
            return rc;
        }
        for (int i = 0; i < n; ++i)
            if (need[i]) scratch[m++] = scratch[i];
        free(need);
    } else {
        for (int i = 0; i < n; ++i) {
            cec_host_update u = scratch[i];
            if (hooks->try_update &&
                !hooks->try_update(lid, u.addr, (char *)(uintptr_t)u.buf, u.len, hooks->ctx))
                continue;
            scratch[m++] = u;
        }
    }
    if (m == 0) return 0;
    rc = cec_drainer_apply(drainer, scratch, m, parity, stream);
    return rc < 0 ? rc : m;
}
