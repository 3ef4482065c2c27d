/*
 * integration/cocytus_recovery_pool.c -- the parity's online recovery coalesced onto a
 * cec_recovery_pool (see cocytus_recovery_pool.h).  Server-side glue: compiled in the
 * Cocytus tree against its own recovery.h (struct recovery / recovery_unit /
 * recovery_queue_item, /root/reference/recovery.h:51-81).
 *
 * The unit flags are the reference's bits (recovery.h:32-48), kept exactly as recovery.c
 * keeps them; a request's units are in at most one request at a time (do_recovery takes
 * sub_flags 0 -> 1, recovery_req_add), so the pool's per-request state (touched, peers
 * contributed) mirrors the per-unit flags of its units, and the pool's fold rule is the
 * per-unit rule of recovery.c:116-120.
 */
#include "cocytus_recovery_pool.h"

#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#define UNIT ((uint64_t)UNITSIZE) /* const.h:26 */
#define F_UPDATE (1u << 30)
#define F_RECOVERED (1u << 31)
#define F_LID(l) (1u << (l))
#define MAT(g, x, y) ((g)->matrix[(x) * (g)->k + (y)]) /* MATRIX(x, y), memcached.h:52 */

enum { kNoSlots = -2 }; /* a request whose mask lacks this parity: nothing to fold here */

struct rq_state {
    int id;     /* pool request, kNoSlots, or -1: not begun */
    int want;   /* a solve is queued */
    int solved; /* the queued solve ran */
    int n_lost;
    int on_pool; /* single loss led by this parity: solved by the pool into its output */
    const struct recovery_queue_item *it;
    char *own[32]; /* the other masks' data[x], malloc'd by the flush */
};

struct cocytus_rpool {
    int k, m, self;
    int *matrix;
    void *stream;
    cec_recovery_pool *pool;
    int qcap;
    struct rq_state *q;
    int *want; /* queue slots with a queued solve, in solve order */
    int n_want;
    cec_region_job *jobs;
    int cap_jobs;
    cec_host_update *win; /* a drain window's updates that fold */
    int cap_win;
    int *win_units; /* [units folded per update | units expected] */
    int cap_win_units;
};

static int grow(void **p, int *cap, int need, size_t elem) {
    if (need <= *cap) return CEC_OK;
    int c = *cap ? *cap : 256;
    while (c < need) c *= 2;
    void *q = realloc(*p, (size_t)c * elem);
    if (!q) return CEC_ENOMEM;
    *p = q;
    *cap = c;
    return CEC_OK;
}

int cocytus_rpool_create(cocytus_rpool **out, int k, int m, const int *matrix, int self_lid, const void *parity_dev,
                         int queue_cap, int capacity_units, void *stream) {
    if (!out || !matrix || k < 1 || m < 1 || k + m > 32 || self_lid < k || self_lid >= k + m || queue_cap < 1)
        return CEC_EINVAL;
    *out = NULL;
    cocytus_rpool *g = calloc(1, sizeof *g);
    if (!g) return CEC_ENOMEM;
    g->matrix = malloc(sizeof(int) * (size_t)((k + m) * k));
    g->q = calloc((size_t)queue_cap, sizeof *g->q);
    g->want = malloc(sizeof(int) * (size_t)queue_cap);
    if (!g->matrix || !g->q || !g->want) {
        cocytus_rpool_destroy(g);
        return CEC_ENOMEM;
    }
    memcpy(g->matrix, matrix, sizeof(int) * (size_t)((k + m) * k));
    g->k = k;
    g->m = m;
    g->self = self_lid;
    g->stream = stream;
    g->qcap = queue_cap;
    for (int i = 0; i < queue_cap; ++i) g->q[i].id = -1;
    const int rc = cec_recovery_pool_create(&g->pool, k, m, matrix, self_lid, (const uint8_t *)parity_dev,
                                            capacity_units);
    if (rc) {
        cocytus_rpool_destroy(g);
        return rc;
    }
    *out = g;
    return CEC_OK;
}

static void free_own(struct rq_state *st) {
    for (int x = 0; x < 32; ++x) {
        free(st->own[x]);
        st->own[x] = NULL;
    }
}

void cocytus_rpool_destroy(cocytus_rpool *g) {
    if (!g) return;
    if (g->q)
        for (int i = 0; i < g->qcap; ++i) free_own(&g->q[i]);
    if (g->pool) cec_recovery_pool_destroy(g->pool);
    free(g->jobs);
    free(g->win);
    free(g->win_units);
    free(g->want);
    free(g->q);
    free(g->matrix);
    free(g);
}

/* the request's slot in recovery.queue.items (its key here) */
static struct rq_state *state_of(cocytus_rpool *g, const struct recovery *r, const struct recovery_queue_item *it) {
    if (!g || !r || !r->units || !it || !r->queue.items) return NULL;
    const ptrdiff_t qi = it - r->queue.items;
    if (qi < 0 || qi >= g->qcap || it->unit_begin < 0 || it->unit_end < it->unit_begin) return NULL;
    return &g->q[qi];
}

int cocytus_rpool_begin(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit) {
    struct rq_state *st = state_of(g, r, rqit);
    if (!st || st->id != -1) return CEC_EINVAL;
    if (!(rqit->mask & F_LID(g->self))) { /* start_fast_recovery's masks: C all from other parities */
        st->id = kNoSlots;
    } else {
        const int id = cec_recovery_pool_begin(g->pool, rqit->mask, rqit->unit_begin, rqit->unit_end);
        if (id < 0) return id;
        st->id = id;
    }
    st->want = st->solved = st->n_lost = st->on_pool = 0;
    st->it = rqit;
    return CEC_OK;
}

static void unqueue(cocytus_rpool *g, int qi) {
    for (int i = 0; i < g->n_want; ++i)
        if (g->want[i] == qi) {
            memmove(g->want + i, g->want + i + 1, sizeof(int) * (size_t)(g->n_want - i - 1));
            g->n_want--;
            return;
        }
}

int cocytus_rpool_end(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit) {
    struct rq_state *st = state_of(g, r, rqit);
    if (!st) return CEC_EINVAL;
    if (st->id == -1) return CEC_OK;
    int rc = CEC_OK;
    if (st->id >= 0) rc = cec_recovery_pool_end(g->pool, st->id);
    if (st->want) unqueue(g, (int)(st - g->q));
    free_own(st);
    memset(st, 0, sizeof *st);
    st->id = -1;
    return rc;
}

int cocytus_rpool_recover_units(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit,
                                int peerid, const char *data) {
    struct rq_state *st = state_of(g, r, rqit);
    if (!st || st->id < 0 || !data || peerid < 0 || peerid >= g->k) return CEC_EINVAL;
    for (int i = rqit->unit_begin; i <= rqit->unit_end; ++i) {
        const struct recovery_unit *u = &r->units[i];
        if (u->flags & F_RECOVERED) return CEC_EINVAL;   /* recovery.c:72 */
        if (u->flags & F_LID(peerid)) return CEC_EINVAL; /* :74 */
        if (u->data) return CEC_EINVAL;                  /* :78; this placement never holds unit->data */
    }
    const int rc = cec_recovery_pool_add_peer(g->pool, st->id, peerid, data); /* :79-93, queued */
    if (rc) return rc;
    for (int i = rqit->unit_begin; i <= rqit->unit_end; ++i) { /* :84-89 */
        struct recovery_unit *u = &r->units[i];
        if (!(u->flags & F_UPDATE)) u->flags |= F_UPDATE | F_LID(g->self);
        u->flags |= F_LID(peerid);
    }
    return CEC_OK;
}

char *cocytus_rpool_staging(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit, int peerid) {
    struct rq_state *st = state_of(g, r, rqit);
    if (!st || st->id < 0) return NULL;
    return (char *)cec_recovery_pool_staging(g->pool, st->id, peerid, NULL);
}

/* recovery_try_update_unit's walk (recovery.c:105-129): the return value, touch_flags, the
 * unit pieces it would fold (*nfold) and the pieces on units under recovery (*nupd) */
static int walk(const cocytus_rpool *g, const struct recovery *r, char *touch_flags, const char *sub_flags,
                int peerid, uint64_t addr, uint32_t size, int *nfold, int *nupd) {
    int ret = 0;
    *nfold = *nupd = 0;
    while (size > 0) {
        const uint64_t offset = addr % UNIT;
        const uint64_t base = addr - offset;
        uint32_t len = (uint32_t)(UNIT - offset);
        if (size < len) len = size;
        size -= len;
        if (touch_flags) touch_flags[base / UNIT] = 1;               /* :112 */
        if (sub_flags == NULL || sub_flags[base / UNIT] != 2) ret++; /* :113 */
        const uint32_t f = r->units[base / UNIT].flags;
        if (!(f & F_RECOVERED) && (f & F_UPDATE) && !(f & F_LID(peerid))) ++*nfold; /* :116-120 */
        if (f & F_UPDATE) ++*nupd;
        addr += len;
    }
    (void)g;
    return ret;
}

/* The fold, before the caller applies the diff to the parity arena (memcached.c:7758-7767).
 * A queued reply's first-touch copy reads the arena at the flush, the reference's at the
 * reply (recovery.c:81): so the queue is flushed before any apply that reaches a unit under
 * recovery (fold_update flushes first itself). */
static int fold(cocytus_rpool *g, int peerid, uint64_t addr, const char *data, uint32_t size, int nfold, int nupd) {
    if (!nfold) {
        const int rc = nupd ? cec_recovery_pool_flush(g->pool, g->stream) : CEC_OK;
        return rc < 0 ? rc : CEC_OK;
    }
    const int folded = cec_recovery_pool_fold_update(g->pool, peerid, addr, data, size, g->stream);
    if (folded < 0) return folded;
    return folded == nfold ? CEC_OK : CEC_EINVAL; /* the pool's requests and the flags disagree */
}

int cocytus_rpool_try_update_unit(cocytus_rpool *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                                  int peerid, uint64_t addr, const char *data, uint32_t size) {
    if (!g || !r || !r->units || peerid < 0 || peerid >= g->k || (size && !data)) return CEC_EINVAL;
    int nfold, nupd;
    const int ret = walk(g, r, touch_flags, sub_flags, peerid, addr, size, &nfold, &nupd);
    const int rc = fold(g, peerid, addr, data, size, nfold, nupd);
    return rc ? rc : ret;
}

int cocytus_rpool_try_update_units(cocytus_rpool *g, struct recovery *r, char *const *touch_flags,
                                   const char *sub_flags, const cec_host_update *u, int n, int *need) {
    if (!g || !r || !r->units || n < 0 || (n && (!u || !need))) return CEC_EINVAL;
    for (int i = 0; i < n; ++i)
        if (u[i].src_lid >= (uint32_t)g->k || (u[i].len && !u[i].buf)) return CEC_EINVAL;
    /* the walks in xid order (the flags do not change within the window), then every fold of
     * the window in one pool call: the applies come after the whole window, so one flush of
     * the queued first touches ahead of them is enough */
    int rc, nf = 0, any_upd = 0;
    if ((rc = grow((void **)&g->win, &g->cap_win, n, sizeof *g->win)) ||
        (rc = grow((void **)&g->win_units, &g->cap_win_units, 2 * n, sizeof *g->win_units)))
        return rc;
    int *want = g->win_units + n;
    for (int i = 0; i < n; ++i) {
        const int lid = (int)u[i].src_lid;
        int nfold, nupd;
        need[i] = walk(g, r, touch_flags ? touch_flags[lid] : NULL, sub_flags, lid, u[i].addr, u[i].len, &nfold,
                       &nupd);
        any_upd |= nupd > 0;
        if (nfold) {
            g->win[nf] = u[i];
            want[nf++] = nfold;
        }
    }
    if (!nf) {
        rc = any_upd ? cec_recovery_pool_flush(g->pool, g->stream) : CEC_OK;
        return rc < 0 ? rc : CEC_OK;
    }
    rc = cec_recovery_pool_fold_updates(g->pool, g->win, nf, g->win_units, g->stream);
    if (rc < 0) return rc;
    for (int i = 0; i < nf; ++i)
        if (g->win_units[i] != want[i]) return CEC_EINVAL; /* the pool's requests and the flags disagree */
    return CEC_OK;
}

int cocytus_rpool_fold_hook(const cec_host_update *u, int n, int *need, void *ctx) {
    cocytus_rpool_fold_ctx *f = ctx;
    if (!f) return CEC_EINVAL;
    return cocytus_rpool_try_update_units(f->g, f->r, f->touch_flags, f->sub_flags, u, n, need);
}

int cocytus_rpool_residual(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit, char *buf) {
    struct rq_state *st = state_of(g, r, rqit);
    if (!st || st->id < 0 || !buf) return CEC_EINVAL;
    return cec_recovery_pool_residual(g->pool, st->id, buf, g->stream);
}

/* memcached.c:7848-7908: lost data lids, the parities of the mask, inv; 0 or a status */
static int split(const cocytus_rpool *g, uint32_t mask, int *lost, int *pars, int *n, int *inv) {
    int nl = 0, np = 0;
    for (int i = 0; i < g->k; ++i)
        if (!(mask & F_LID(i))) lost[nl++] = i;
    for (int i = g->k; i < g->k + g->m; ++i)
        if (mask & F_LID(i)) pars[np++] = i;
    if (np != nl) return CEC_EINVAL; /* :7891 assert(m == n) */
    *n = nl;
    if (!nl) return CEC_OK;
    int tmp[32 * 32], t = 0;
    for (int p = 0; p < nl; ++p)
        for (int x = 0; x < nl; ++x) tmp[t++] = MAT(g, pars[p], lost[x]);
    return jerasure_invert_matrix(tmp, inv, nl, 8) == 0 ? CEC_OK : CEC_ESINGULAR; /* :7907-7908 */
}

int cocytus_rpool_solve(cocytus_rpool *g, struct recovery *r, const struct recovery_queue_item *rqit, int *n_out) {
    struct rq_state *st = state_of(g, r, rqit);
    if (!st || st->id == -1 || !n_out || st->want) return CEC_EINVAL;
    int lost[32], pars[32], n, inv[32 * 32];
    int rc = split(g, rqit->mask, lost, pars, &n, inv);
    if (rc) return rc;
    if (!n) {
        *n_out = 0;
        return CEC_OK;
    }
    for (int p = 0; p < n; ++p) {
        if (pars[p] == g->self) {
            if (st->id < 0 || !cec_recovery_pool_complete(g->pool, st->id)) return CEC_EINVAL;
        } else if (!rqit->data_from_parity || !rqit->data_from_parity[pars[p]]) {
            return CEC_EINVAL;
        }
    }
    free_own(st);
    st->want = 1;
    st->solved = 0;
    st->n_lost = n;
    st->on_pool = n == 1 && pars[0] == g->self;
    st->it = rqit;
    g->want[g->n_want++] = (int)(st - g->q);
    *n_out = n;
    return CEC_OK;
}

int cocytus_rpool_pending(const cocytus_rpool *g) { return g ? g->n_want : 0; }

/* The masks the pool does not solve: data[x] = sum_p inv[x][p] * C[p] over host buffers,
 * C[self] read back from the pool, all of them in one batch. */
static int solve_on_host(cocytus_rpool *g) {
    int nj = 0, rc = CEC_OK, n_cself = 0;
    char **cself = calloc((size_t)g->n_want + 1, sizeof *cself); /* this parity's C, one per request */
    if (!cself) return CEC_ENOMEM;
    for (int w = 0; w < g->n_want && !rc; ++w) {
        struct rq_state *st = &g->q[g->want[w]];
        if (st->on_pool) continue;
        const struct recovery_queue_item *it = st->it;
        const uint64_t nbuf = (uint64_t)(it->unit_end - it->unit_begin + 1) * UNIT;
        int lost[32], pars[32], n, inv[32 * 32];
        if ((rc = split(g, it->mask, lost, pars, &n, inv))) break;
        if (nbuf > UINT32_MAX) {
            rc = CEC_EINVAL;
            break;
        }
        const char *C[32];
        for (int p = 0; p < n && !rc; ++p) {
            if (pars[p] != g->self) {
                C[p] = it->data_from_parity[pars[p]];
                continue;
            }
            char *b = malloc(nbuf); /* memcached.c:7856-7864: this parity's units */
            if (!b) {
                rc = CEC_ENOMEM;
                break;
            }
            cself[n_cself++] = b;
            rc = cec_recovery_pool_residual(g->pool, st->id, b, g->stream);
            C[p] = b;
        }
        if (rc || (rc = grow((void **)&g->jobs, &g->cap_jobs, nj + n * n, sizeof *g->jobs))) break;
        for (int x = 0; x < n && !rc; ++x)
            if (!(st->own[x] = malloc(nbuf))) rc = CEC_ENOMEM;
        for (int x = 0; x < n && !rc; ++x)
            for (int p = 0; p < n; ++p) { /* :7916-7922; the first term writes (calloc + ^=) */
                cec_region_job *j = &g->jobs[nj++];
                j->src = C[p];
                j->dst = st->own[x];
                j->base = NULL;
                j->len = (uint32_t)nbuf;
                j->multby = inv[x * n + p];
                j->add = p > 0;
            }
    }
    if (!rc && nj) rc = cec_region_multiply_batch(g->jobs, nj, g->stream);
    for (int i = 0; i < n_cself; ++i) free(cself[i]);
    free(cself);
    return rc;
}

int cocytus_rpool_flush(cocytus_rpool *g) {
    if (!g) return CEC_EINVAL;
    /* one launch: every queued reply folded, every single-loss request it completes solved */
    int rc = cec_recovery_pool_flush_solve_host(g->pool, g->stream);
    if (rc < 0) return rc;
    int ids[1024], n = 0;
    for (int w = 0; w < g->n_want; ++w) { /* requests completed before this pass: solved now */
        const struct rq_state *st = &g->q[g->want[w]];
        if (!st->on_pool || cec_recovery_pool_solved(g->pool, st->id)) continue;
        ids[n++] = st->id;
        if (n == 1024) {
            if ((rc = cec_recovery_pool_solve_host(g->pool, ids, n, g->stream))) return rc;
            n = 0;
        }
    }
    if (n && (rc = cec_recovery_pool_solve_host(g->pool, ids, n, g->stream))) return rc;
    if ((rc = solve_on_host(g))) return rc;
    const int done = g->n_want;
    for (int w = 0; w < g->n_want; ++w) {
        struct rq_state *st = &g->q[g->want[w]];
        st->want = 0;
        st->solved = 1;
    }
    g->n_want = 0;
    return done;
}

const char *cocytus_rpool_data(const cocytus_rpool *g, const struct recovery *r, const struct recovery_queue_item *rqit,
                               int x) {
    const struct rq_state *st = state_of((cocytus_rpool *)g, r, rqit);
    if (!st || !st->solved || x < 0 || x >= st->n_lost) return NULL;
    if (st->on_pool) return (const char *)cec_recovery_pool_output(g->pool, st->id, NULL);
    return st->own[x];
}
