/*
 * tests/glue/cluster_sim.c -- an RS(K,M) Cocytus group replayed in one process through the
 * server glue (integration/cocytus_{set,drain,recovery}.c) over the server's own types
 * (rep_queue.h, recovery.h, ecmem.h where they lie), to check the glue end to end against
 * the one truth that needs no oracle: the bytes a lost data shard held.
 *
 *   cluster_sim SEED [DEFER [CONTROL [NLOST_MAX]]]   (NLOST_MAX: at most this many data lids lost, <= M)
 *
 * DEFER: 0 the immediate glue calls, 1 the deferred ones (cocytus_recovery.c, both), 2 the pool
 * placement (cocytus_recovery_pool.c: the residuals in a cec_recovery_pool per parity, replies
 * copied or received into its staging, the non-leaders' units sent from cocytus_rpool_residual,
 * the leader's solve at cocytus_rpool_flush; unit->data stays NULL).
 *
 * CONTROL = 1 breaks the protocol on purpose (a reply applied before its peer's queued diffs
 * are drained): the rebuilt bytes must then differ -- the check has teeth.
 *
 * K data processes and M parity processes, host arenas (ecmem) of NU units each:
 *   SET      a data process computes diff = new ^ old (cocytus_set_diffs_gf, memcached.c:
 *            2664-2681), installs the value (:5663-5666) and queues the diff at every parity
 *            under its next xid (rep_queue_add; parity_send);
 *   drain    a parity drains a data lid's queue up to its newest xid: cocytus_drain_gf with
 *            the recovery glue's fold hook into its arena, registered with cec_host_register
 *            (memcached.c:4231 / 4322 / 4350 -> process_rep_command :7739-7798), then frees
 *            the entries as rep_queue_flush does;
 *   failure  data lid LOST stops; its arena at that moment is the truth;
 *   recovery the leader parity recovers unit ranges (start_recovery's mask: itself + the K-1
 *            surviving data lids, memcached.c:8136-8151).  Each surviving peer's reply is its
 *            arena's bytes of the range; before applying it the leader drains that peer's
 *            queue (recover_units_reply, :4311-4316), then cocytus_recover_units_gf (or the
 *            deferred form); SETs keep arriving from the survivors throughout, and the
 *            leader drains at random moments, folding them into the units where
 *            recovery_try_update_unit would (recovery.c:99-131).  When every reply is in,
 *            cocytus_recovery_solve_gf rebuilds the range (memcached.c:7842-7922).
 * Checks: every rebuilt range equals the lost shard's bytes; at the end every parity arena
 * equals sum_j MATRIX(p, j) * D_j of the data arenas (the oracle's region multiply, on the
 * host).  Prints "ok ranges N sets S folds F" or the first mismatch; exit status 0 / 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cocytus_ec.h>

#include "cocytus_drain.h"
#include "cocytus_recovery.h"
#include "cocytus_recovery_pool.h"
#include "cocytus_set.h"
#include "gf8_ref.h" /* oracle: the final parity check only */
#include "rep_queue.h"

#ifndef K /* the code: -DK= -DM= (default RS(3,2)) */
#define K 3
#endif
#ifndef M
#define M 2
#endif
#define NU 512 /* units per arena: 2 MiB */
#define U ((size_t)UNITSIZE)
#define QCAP 4096

static uint64_t rng_s;
static uint64_t rnd(void) {
    rng_s ^= rng_s << 13, rng_s ^= rng_s >> 7, rng_s ^= rng_s << 17;
    return rng_s;
}

struct parity {
    int lid;
    struct ecmem ecm;
    uint8_t *dev; /* registered alias */
    struct rep_queue q[K];
    uint64_t done[K];
    uint32_t nbytes[K][QCAP];
    struct recovery rec;
    char *touch[K + M];
    cocytus_rglue *g;
    cocytus_fold_ctx fold;
    cec_drainer *dr;
    cocytus_rpool *pg; /* DEFER 2 */
    cocytus_rpool_fold_ctx pfold;
    struct recovery_queue_item item[1]; /* rec.queue.items: one request in flight */
};

static int pool_mode;

static int *matrix;
static struct ecmem data[K];
static struct parity par[M];
static uint64_t next_xid[K];
static int sets;

static uint32_t item_nbytes(void *item, void *ctx) {
    (void)ctx;
    return *(uint32_t *)item;
}

static int drain(struct parity *p, int lid, int defer) {
    struct rep_queue *q = &p->q[lid];
    const uint64_t upto = next_xid[lid] - 1;
    if (p->done[lid] >= upto) return 0;
    static cec_host_update scratch[QCAP];
    p->fold.defer = defer;
    cocytus_drain_hooks hooks = {.item_nbytes = item_nbytes, .try_update_batch = cocytus_fold_hook, .ctx = &p->fold};
    if (pool_mode) {
        hooks.try_update_batch = cocytus_rpool_fold_hook;
        hooks.ctx = &p->pfold;
    }
    const int rc = cocytus_drain_gf(q, lid, p->done[lid], upto, &hooks, p->dr, p->dev, NULL, scratch, QCAP);
    if (rc < 0) {
        fprintf(stderr, "drain: %d %s\n", rc, cec_last_error());
        exit(2);
    }
    /* process_rep_command's tail per xid (done) and rep_queue_flush (free the vbufs) */
    while (q->tail != q->head) {
        struct rep_queue_item *e = &q->items[q->tail % q->cap];
        free(e->vbuf);
        e->vbuf = NULL;
        q->tail++;
    }
    p->done[lid] = upto;
    return rc;
}

/* the ring's add as rep_queue_add does it (rep_queue.c:48-61; rep_queue.c itself needs
 * memcached.h and <event.h>, so the test keeps its own) */
static struct rep_queue_item *sim_queue_add(struct rep_queue *q) {
    if (q->head - q->tail == q->cap) return NULL;
    if (q->tail > q->cap) {
        q->tail -= q->cap;
        q->head -= q->cap;
    }
    struct rep_queue_item *e = &q->items[q->head % q->cap];
    e->ack = 0;
    q->head++;
    return e;
}

static void set(int j, int defer_unused) {
    (void)defer_unused;
    const uint32_t len = 1 + (uint32_t)(rnd() % (3 * U));
    const uint64_t addr = 16 * (rnd() % ((NU * U - len) / 16));
    char *value = malloc(len), *diff = malloc(len + 16);
    for (uint32_t b = 0; b < len; ++b) value[b] = (char)rnd();
    cocytus_set_diff sd = {value, addr, len, diff};
    if (cocytus_set_diffs_gf(&data[j], &sd, 1, NULL)) {
        fprintf(stderr, "set diff: %s\n", cec_last_error());
        exit(2);
    }
    memcpy((char *)data[j].mem + addr, value, len); /* install (memcached.c:5663-5666) */
    const uint64_t xid = next_xid[j]++;
    for (int p = 0; p < M; ++p) { /* parity_send to every parity */
        struct rep_queue *q = &par[p].q[j];
        if (q->head - q->tail >= q->cap) drain(&par[p], j, 0);
        struct rep_queue_item *e = sim_queue_add(q);
        if (!e) exit(3);
        e->xid = xid;
        e->lid = j;
        e->addr = addr;
        e->vbuf = malloc(len);
        memcpy(e->vbuf, diff, len);
        e->vnbytes = (int)len;
        par[p].nbytes[j][(q->head - 1) % q->cap] = len;
        e->item = &par[p].nbytes[j][(q->head - 1) % q->cap];
        e->done = 0;
    }
    free(value);
    free(diff);
    sets++;
}

int main(int argc, char **argv) {
    if (argc < 2) return 1;
    const uint64_t seed = (uint64_t)atoll(argv[1]);
    rng_s = 0x9E3779B97F4A7C15ull ^ seed * 0x2545F4914F6CDD1Dull;
    const int defer = argc > 2 ? atoi(argv[2]) : 0;
    pool_mode = defer == 2;
    const int control = argc > 3 && atoi(argv[3]);
    const int nlost_max = argc > 4 ? atoi(argv[4]) : M;
    if (nlost_max < 1) return 1;
    if (cec_device_check() != CEC_OK) return fprintf(stderr, "%s\n", cec_last_error()), 2;
    matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    for (int j = 0; j < K; ++j) { /* the data processes' ecmem, registered (SET diffs read the
                                     old bytes in place) */
        data[j].size = NU * U;
        if (posix_memalign(&data[j].mem, 4096, NU * U)) return 2;
        memset(data[j].mem, 0, NU * U);
        uint8_t *alias;
        if (cec_host_register(data[j].mem, NU * U, &alias)) return fprintf(stderr, "%s\n", cec_last_error()), 2;
        next_xid[j] = 1;
    }
    for (int p = 0; p < M; ++p) {
        struct parity *P = &par[p];
        P->lid = K + p;
        P->ecm.size = NU * U;
        if (posix_memalign(&P->ecm.mem, 4096, NU * U)) return 2;
        memset(P->ecm.mem, 0, NU * U);
        if (cec_host_register(P->ecm.mem, NU * U, &P->dev)) return fprintf(stderr, "%s\n", cec_last_error()), 2;
        for (int j = 0; j < K; ++j) {
            P->q[j].cap = QCAP;
            P->q[j].items = calloc(QCAP, sizeof(struct rep_queue_item));
        }
        P->rec.units = calloc(NU, sizeof(struct recovery_unit));
        for (int l = 0; l < K + M; ++l) P->touch[l] = calloc(NU, 1);
        if (cocytus_rglue_create(&P->g, K, M, matrix, P->lid, NULL) ||
            cec_drainer_create(&P->dr, K, M, matrix, P->lid, 8 << 20))
            return 2;
        P->fold.g = P->g;
        P->fold.r = &P->rec;
        for (int l = 0; l < K + M; ++l) P->fold.touch_flags[l] = P->touch[l];
        P->fold.sub_flags = NULL;
        P->rec.queue.items = P->item;
        P->rec.queue.cap = 1;
        if (pool_mode && cocytus_rpool_create(&P->pg, K, M, matrix, P->lid, P->dev, 1, 32, NULL))
            return fprintf(stderr, "rpool: %s\n", cec_last_error()), 2;
        P->pfold.g = P->pg;
        P->pfold.r = &P->rec;
        for (int l = 0; l < K + M; ++l) P->pfold.touch_flags[l] = P->touch[l];
        P->pfold.sub_flags = NULL;
    }
    /* normal operation: SETs everywhere, drains now and then */
    for (int i = 0; i < 600; ++i) {
        set((int)(rnd() % K), 0);
        if (rnd() % 8 == 0) drain(&par[rnd() % M], (int)(rnd() % K), 0);
    }
    for (int p = 0; p < M; ++p)
        for (int j = 0; j < K; ++j) drain(&par[p], j, 0);
    /* NL data lids fail (1 <= NL <= M): their arenas are the truth.  The leader parity
     * recovers ranges with start_recovery's mask (memcached.c:8136-8151: itself, then the
     * first K-1 connected lids in lid order -- the surviving data lids, then other
     * parities); every parity of the mask folds the survivors' replies (recover_units_reply
     * goes to each, :4277-4282) and the non-leaders ship their units to the leader
     * (send_recovered_data, :7822-7834, into rqit->data_from_parity) before it solves. */
    const int nl = 1 + (int)(seed % (uint64_t)(nlost_max < M ? nlost_max : M)); /* every count over the seeds */
    int lost[M], is_lost[K] = {0};
    for (int x = 0; x < nl;) {
        const int j = (int)(rnd() % K);
        if (!is_lost[j]) is_lost[j] = 1, x++;
    }
    for (int j = 0, x = 0; j < K; ++j)
        if (is_lost[j]) lost[x++] = j;
    struct parity *L = &par[rnd() % M];
    uint32_t mask = 1u << L->lid;
    for (int i = 0, remaining = K - 1; i < K + M && remaining; ++i) {
        if (i == L->lid || (i < K && is_lost[i])) continue;
        mask |= 1u << i;
        remaining--;
    }
    struct parity *part[M];
    int np = 0;
    for (int p = 0; p < M; ++p)
        if (mask & (1u << par[p].lid)) part[np++] = &par[p];
    int ranges = 0, bad = 0;
    for (int ub = 0; ub < NU && !bad;) {
        const int span = (int)(rnd() % 24);
        const int ue = ub + span < NU - 1 ? ub + span : NU - 1;
        const size_t nbuf = (size_t)(ue - ub + 1) * U;
        char *dfp[K + M];
        memset(dfp, 0, sizeof dfp);
        for (int q = 0; q < np && pool_mode; ++q) { /* recovery_req_add at each parity of the mask */
            struct recovery_queue_item *it = &part[q]->item[0];
            memset(it, 0, sizeof *it);
            it->unit_begin = ub;
            it->unit_end = ue;
            it->mask = mask;
            it->in_use = 1;
            it->data_from_parity = dfp;
            if (cocytus_rpool_begin(part[q]->pg, &part[q]->rec, it))
                return fprintf(stderr, "begin: %s\n", cec_last_error()), 2;
        }
        /* replies arrive in a random order, SETs and drains before, between and after */
        int order[K], no = 0;
        for (int j = 0; j < K; ++j)
            if (!is_lost[j]) order[no++] = j;
        for (int x = no - 1; x > 0; --x) {
            const int y = (int)(rnd() % (uint64_t)(x + 1)), t = order[x];
            order[x] = order[y];
            order[y] = t;
        }
        for (int r = 0; r <= no; ++r) {
            const int burst = (int)(rnd() % 12);
            for (int i = 0; i < burst; ++i) {
                int j;
                do j = (int)(rnd() % K);
                while (is_lost[j]);
                set(j, 0);
                if (rnd() % 3 == 0) drain(part[rnd() % np], j, defer); /* folds into the units */
            }
            if (r == no) break;
            const int peer = order[r];
            for (int q = 0; q < np; ++q) { /* each parity of the mask gets the reply */
                struct parity *P = part[q];
                if (!control) drain(P, peer, defer); /* recover_units_reply: the peer's xids first (:4311-4316) */
                if (pool_mode) { /* received into the pool's staging, or copied in from c->vbuf */
                    char *st = rnd() % 2 ? cocytus_rpool_staging(P->pg, &P->rec, &P->item[0], peer) : NULL;
                    char *reply = st ? st : malloc(nbuf);
                    memcpy(reply, (char *)data[peer].mem + (size_t)ub * U, nbuf);
                    const int rc = cocytus_rpool_recover_units(P->pg, &P->rec, &P->item[0], peer, reply);
                    if (!st) free(reply);
                    if (rc) return fprintf(stderr, "recover: %d %s\n", rc, cec_last_error()), 2;
                    continue;
                }
                char *reply = malloc(nbuf);
                memcpy(reply, (char *)data[peer].mem + (size_t)ub * U, nbuf);
                const int rc = defer ? cocytus_recover_units_defer(P->g, &P->rec, &P->ecm, peer, ub, ue, reply, 1)
                                     : cocytus_recover_units_gf(P->g, &P->rec, &P->ecm, peer, ub, ue, reply);
                if (!defer) free(reply);
                if (rc) return fprintf(stderr, "recover: %d %s\n", rc, cec_last_error()), 2;
            }
        }
        if (pool_mode) { /* non-leaders send their residuals, the leader solves at its flush */
            for (int q = 0; q < np; ++q) {
                struct parity *P = part[q];
                if (P == L) continue;
                dfp[P->lid] = malloc(nbuf);
                if (cocytus_rpool_residual(P->pg, &P->rec, &P->item[0], dfp[P->lid]))
                    return fprintf(stderr, "residual: %s\n", cec_last_error()), 2;
            }
            int n = 0;
            if (cocytus_rpool_solve(L->pg, &L->rec, &L->item[0], &n) || n != nl || cocytus_rpool_flush(L->pg) != 1)
                return fprintf(stderr, "solve: n %d of %d: %s\n", n, nl, cec_last_error()), 2;
            for (int x = 0; x < n; ++x) {
                const char *d = cocytus_rpool_data(L->pg, &L->rec, &L->item[0], x);
                if ((!d || memcmp(d, (char *)data[lost[x]].mem + (size_t)ub * U, nbuf)) && !bad) {
                    printf("range [%d, %d]: rebuilt bytes of lid %d differ from the lost shard\n", ub, ue, lost[x]);
                    bad = 1;
                }
            }
            for (int l = 0; l < K + M; ++l) free(dfp[l]);
            for (int q = 0; q < np; ++q) { /* recovery_req_remove: the glue first (recovery.c:196-205) */
                if (cocytus_rpool_end(part[q]->pg, &part[q]->rec, &part[q]->item[0]))
                    return fprintf(stderr, "end: %s\n", cec_last_error()), 2;
                for (int i = ub; i <= ue; ++i) part[q]->rec.units[i].flags = 0;
            }
            ranges++;
            ub = ue + 1;
            continue;
        }
        struct recovery_queue_item it;
        memset(&it, 0, sizeof it);
        it.unit_begin = ub;
        it.unit_end = ue;
        it.mask = mask;
        it.data_from_parity = dfp;
        for (int q = 0; q < np; ++q) {
            struct parity *P = part[q];
            if (defer && cocytus_recovery_flush(P->g) < 0) return fprintf(stderr, "flush: %s\n", cec_last_error()), 2;
            if (P == L) continue;
            dfp[P->lid] = malloc(nbuf); /* send_recovered_data: its units, in order */
            for (int i = ub; i <= ue; ++i) memcpy(dfp[P->lid] + (size_t)(i - ub) * U, P->rec.units[i].data, U);
        }
        char *out[M];
        int n = 0;
        if (cocytus_recovery_solve_gf(L->g, &L->rec, &it, out, &n) || n != nl)
            return fprintf(stderr, "solve: n %d of %d: %s\n", n, nl, cec_last_error()), 2;
        for (int x = 0; x < n; ++x) {
            if (memcmp(out[x], (char *)data[lost[x]].mem + (size_t)ub * U, nbuf) && !bad) {
                printf("range [%d, %d]: rebuilt bytes of lid %d differ from the lost shard\n", ub, ue, lost[x]);
                bad = 1;
            }
            free(out[x]);
        }
        for (int l = 0; l < K + M; ++l) free(dfp[l]);
        for (int q = 0; q < np; ++q) /* recovery_req_remove (recovery.c:196-205) */
            for (int i = ub; i <= ue; ++i) {
                free(part[q]->rec.units[i].data);
                part[q]->rec.units[i].data = NULL;
                part[q]->rec.units[i].flags = 0;
            }
        ranges++;
        ub = ue + 1;
    }
    /* the parities stayed the code of the data (after draining everything) */
    for (int p = 0; p < M && !bad; ++p) {
        for (int j = 0; j < K; ++j) drain(&par[p], j, 0);
        uint8_t *want = calloc(NU, U);
        for (int j = 0; j < K; ++j)
            ref_region_multiply((uint8_t *)data[j].mem, matrix[(K + p) * K + j], (long)(NU * U), want, 1);
        if (memcmp(want, par[p].ecm.mem, NU * U)) {
            printf("parity %d differs from the encode of the data arenas\n", K + p);
            bad = 1;
        }
        free(want);
    }
    if (!bad) printf("ok RS(%d,%d) ranges %d sets %d lost %d data lids, leader %d\n", K, M, ranges, sets, nl, L->lid);
    for (int j = 0; j < K; ++j) cec_host_unregister(data[j].mem);
    for (int p = 0; p < M; ++p) {
        cocytus_rglue_destroy(par[p].g);
        cocytus_rpool_destroy(par[p].pg);
        cec_drainer_destroy(par[p].dr);
        cec_host_unregister(par[p].ecm.mem);
    }
    return bad;
}
