/*
 * integration/cocytus_recovery.c -- the parity's online-recovery arithmetic batched onto
 * libcocytus_ec (see cocytus_recovery.h).  Server-side glue: compiled in the Cocytus tree
 * against its own recovery.h (struct recovery / recovery_unit / recovery_queue_item,
 * /root/reference/recovery.h:51-81) and ecmem.h.
 *
 * The unit flags are the reference's bits (recovery.h:32-48): bit 30 UPDATE (the unit
 * takes updates during recovery: first touched), bit 31 RECOVERED, bit `lid` = that lid's
 * bytes are in the unit.  They are tested with unsigned masks here (the header's macros
 * shift a signed 1 into bit 31).
 */
#include "cocytus_recovery.h"

#include <stdlib.h>
#include <string.h>

#define UNIT ((uint64_t)UNITSIZE) /* const.h:26 */
#define F_UPDATE (1u << 30)
#define F_RECOVERED (1u << 31)
#define F_LID(l) (1u << (l))

struct cocytus_rglue {
    int k, m, self;
    int *matrix;
    void *stream;
    cec_region_job *tmp; /* immediate calls */
    int cap_tmp;
    cec_region_job *fold; /* deferred folds */
    int n_fold, cap_fold, req_fold;
    cec_region_job *solve; /* deferred solves */
    int n_solve, cap_solve, req_solve;
    char **owned; /* reply buffers freed after the flush */
    int n_owned, cap_owned;
};

#define MAT(g, x, y) ((g)->matrix[(x) * (g)->k + (y)]) /* MATRIX(x, y), memcached.h:52 */

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

int cocytus_rglue_create(cocytus_rglue **out, int k, int m, const int *matrix, int self_lid, void *stream) {
    if (!out || !matrix || k < 1 || m < 1 || k + m > 32 || self_lid < k || self_lid >= k + m) return CEC_EINVAL;
    cocytus_rglue *g = calloc(1, sizeof *g);
    if (!g) return CEC_ENOMEM;
    g->matrix = malloc(sizeof(int) * (size_t)((k + m) * k));
    if (!g->matrix) {
        free(g);
        return CEC_ENOMEM;
    }
    memcpy(g->matrix, matrix, sizeof(int) * (size_t)((k + m) * k));
    g->k = k;
    g->m = m;
    g->self = self_lid;
    g->stream = stream;
    *out = g;
    return CEC_OK;
}

void cocytus_rglue_destroy(cocytus_rglue *g) {
    if (!g) return;
    for (int i = 0; i < g->n_owned; ++i) free(g->owned[i]);
    free(g->owned);
    free(g->tmp);
    free(g->fold);
    free(g->solve);
    free(g->matrix);
    free(g);
}

int cocytus_recovery_pending(const cocytus_rglue *g) { return g ? g->req_fold + g->req_solve : 0; }

/* recovery.c:72-78's assertions over the range, before anything changes */
static int check_units(const cocytus_rglue *g, const struct recovery *r, const struct ecmem *ecm, int peerid,
                       int ubegin, int uend, const char *data) {
    if (!g || !r || !r->units || !ecm || !data || peerid < 0 || peerid >= g->k || ubegin < 0 || uend < ubegin)
        return CEC_EINVAL;
    for (int i = ubegin; i <= uend; ++i) {
        const struct recovery_unit *u = &r->units[i];
        if (u->flags & F_RECOVERED) return CEC_EINVAL;           /* :72 */
        if (u->flags & F_LID(peerid)) return CEC_EINVAL;         /* :74 */
        if (!(u->flags & F_UPDATE) && u->data) return CEC_EINVAL; /* :78 */
        if ((u->flags & F_UPDATE) && !u->data) return CEC_EINVAL;
    }
    return CEC_OK;
}

/* malloc(UNITSIZE) for every first-touched unit (recovery.c:79); all or nothing */
static int alloc_first(struct recovery *r, int ubegin, int uend) {
    for (int i = ubegin; i <= uend; ++i) {
        struct recovery_unit *u = &r->units[i];
        if (u->flags & F_UPDATE) continue;
        u->data = malloc(UNITSIZE);
        if (!u->data) {
            for (int j = ubegin; j < i; ++j)
                if (!(r->units[j].flags & F_UPDATE)) {
                    free(r->units[j].data);
                    r->units[j].data = NULL;
                }
            return CEC_ENOMEM;
        }
    }
    return CEC_OK;
}

static void free_first(struct recovery *r, int ubegin, int uend) {
    for (int i = ubegin; i <= uend; ++i)
        if (!(r->units[i].flags & F_UPDATE)) {
            free(r->units[i].data);
            r->units[i].data = NULL;
        }
}

/* recovery.c:84-89 */
static void set_flags(const cocytus_rglue *g, struct recovery *r, int peerid, int ubegin, int uend) {
    for (int i = ubegin; i <= uend; ++i) {
        struct recovery_unit *u = &r->units[i];
        if (!(u->flags & F_UPDATE)) u->flags |= F_UPDATE | F_LID(g->self);
        u->flags |= F_LID(peerid);
    }
}

int cocytus_recover_units_gf(cocytus_rglue *g, struct recovery *r, struct ecmem *ecm, int peerid, int ubegin,
                             int uend, const char *data) {
    int rc = check_units(g, r, ecm, peerid, ubegin, uend, data);
    if (rc) return rc;
    const int nu = uend - ubegin + 1;
    if ((rc = grow((void **)&g->tmp, &g->cap_tmp, nu, sizeof *g->tmp))) return rc;
    if ((rc = alloc_first(r, ubegin, uend))) return rc;
    const int c = MAT(g, g->self, peerid); /* recovery.c:92 */
    for (int i = ubegin; i <= uend; ++i) {
        const struct recovery_unit *u = &r->units[i];
        cec_region_job *j = &g->tmp[i - ubegin];
        j->src = data + (uint64_t)(i - ubegin) * UNIT;
        j->dst = u->data;
        /* first touch: unit = parity unit ^ c * peer (recovery.c:81 memcpy, then :91) */
        j->base = (u->flags & F_UPDATE) ? NULL : ecmem_get(ecm, (uint64_t)i * UNIT);
        j->len = UNITSIZE;
        j->multby = c;
        j->add = 1;
    }
    rc = cec_region_multiply_batch(g->tmp, nu, g->stream);
    if (rc) {
        free_first(r, ubegin, uend);
        return rc;
    }
    set_flags(g, r, peerid, ubegin, uend);
    return CEC_OK;
}

int cocytus_recover_units_defer(cocytus_rglue *g, struct recovery *r, struct ecmem *ecm, int peerid, int ubegin,
                                int uend, char *data, int take) {
    int rc = check_units(g, r, ecm, peerid, ubegin, uend, data);
    if (rc) return rc;
    const int nu = uend - ubegin + 1;
    if ((rc = grow((void **)&g->fold, &g->cap_fold, g->n_fold + nu, sizeof *g->fold))) return rc;
    if (take && (rc = grow((void **)&g->owned, &g->cap_owned, g->n_owned + 1, sizeof *g->owned))) return rc;
    if ((rc = alloc_first(r, ubegin, uend))) return rc;
    const int c = MAT(g, g->self, peerid);
    for (int i = ubegin; i <= uend; ++i) {
        struct recovery_unit *u = &r->units[i];
        if (!(u->flags & F_UPDATE)) /* the first-touch copy now, as the reply arrives (recovery.c:81) */
            memcpy(u->data, ecmem_get(ecm, (uint64_t)i * UNIT), UNITSIZE);
        cec_region_job *j = &g->fold[g->n_fold++];
        j->src = data + (uint64_t)(i - ubegin) * UNIT;
        j->dst = u->data;
        j->base = NULL;
        j->len = UNITSIZE;
        j->multby = c;
        j->add = 1;
    }
    set_flags(g, r, peerid, ubegin, uend);
    if (take) g->owned[g->n_owned++] = data;
    g->req_fold++;
    return CEC_OK;
}

/* recovery_try_update_unit's walk (recovery.c:105-129) over one update, in two passes so that
 * a refusal changes nothing (cocytus_recovery.h: the reference's checks come first):
 *   check  (commit == 0): no write; CEC_EINVAL if a piece would fold into a unit with UPDATE
 *          set and no data (the reference would dereference NULL at recovery.c:123), else the
 *          number of folds the update makes;
 *   commit (commit != 0): touch_flags set, folds appended at (*jobs)[*n] (the caller grew
 *          the array by the check's count), returns what the reference returns.
 * struct recovery carries no unit count: the unit index is bounded by the server's arena, as
 * in recovery_get_unit. */
static int try_update_walk(const cocytus_rglue *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                           int peerid, uint64_t addr, const char *data, uint32_t size, int commit,
                           cec_region_job *jobs, int *n) {
    int ret = 0, folds = 0;
    const int c = MAT(g, g->self, peerid);
    while (size > 0) {
        const uint64_t offset = addr % UNIT;
        const uint64_t base = addr - offset;
        uint32_t len = (uint32_t)(UNIT - offset);
        if (size < len) len = size;
        size -= len;
        if (commit && touch_flags) touch_flags[base / UNIT] = 1;           /* :112 */
        if (sub_flags == NULL || sub_flags[base / UNIT] != 2) ret++;      /* :113 */
        struct recovery_unit *u = &r->units[base / UNIT];
        /* :116-120: recovered, not taking updates, or this peer's bytes already in */
        if (!(u->flags & F_RECOVERED) && (u->flags & F_UPDATE) && !(u->flags & F_LID(peerid))) {
            if (!u->data) return CEC_EINVAL;
            folds++;
            if (commit) {
                cec_region_job *j = &jobs[(*n)++];
                j->src = data;
                j->dst = u->data + offset;
                j->base = NULL;
                j->len = len;
                j->multby = c;
                j->add = 1;
            }
        }
        addr += len;
        data += len;
    }
    return commit ? ret : folds;
}

/* Both passes over a window of updates (a single update is a window of one): every update
 * checked, then *jobs grown by the folds of all of them, then committed -- a refused window
 * leaves touch_flags, need[] and the queue as they were.  *src_bytes (optional) receives
 * the bytes the folds read. */
static int try_update_window(cocytus_rglue *g, struct recovery *r, char *const *touch_flags, char *touch_one,
                             const char *sub_flags, const cec_host_update *u, int n, int *need,
                             cec_region_job **jobs, int *nj, int *cap) {
    int folds = 0;
    for (int i = 0; i < n; ++i) {
        const int lid = (int)u[i].src_lid;
        const int f = try_update_walk(g, r, NULL, sub_flags, lid, u[i].addr, (const char *)u[i].buf, u[i].len, 0,
                                      NULL, NULL);
        if (f < 0) return f;
        folds += f;
    }
    int rc = grow((void **)jobs, cap, *nj + folds, sizeof **jobs);
    if (rc) return rc;
    int last = 0;
    for (int i = 0; i < n; ++i) {
        const int lid = (int)u[i].src_lid;
        char *tf = touch_flags ? touch_flags[lid] : touch_one;
        last = try_update_walk(g, r, tf, sub_flags, lid, u[i].addr, (const char *)u[i].buf, u[i].len, 1, *jobs, nj);
        if (need) need[i] = last;
    }
    return last;
}

/* one update as a window of one */
static cec_host_update one_update(int peerid, uint64_t addr, const char *data, uint32_t size) {
    cec_host_update x;
    x.buf = data;
    x.addr = addr;
    x.len = size;
    x.src_lid = (uint32_t)peerid;
    return x;
}

int cocytus_try_update_unit_gf(cocytus_rglue *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                               int peerid, uint64_t addr, const char *data, uint32_t size) {
    if (!g || !r || !r->units || peerid < 0 || peerid >= g->k || (size && !data)) return CEC_EINVAL;
    const cec_host_update x = one_update(peerid, addr, data, size);
    int n = 0;
    const int ret = try_update_window(g, r, NULL, touch_flags, sub_flags, &x, 1, NULL, &g->tmp, &n, &g->cap_tmp);
    if (ret < 0) return ret;
    if (n) {
        const int rc = cec_region_multiply_batch(g->tmp, n, g->stream);
        if (rc) return rc;
    }
    return ret;
}

static int check_window(const cocytus_rglue *g, const struct recovery *r, const cec_host_update *u, int n, int *need) {
    if (!g || !r || !r->units || n < 0 || (n && (!u || !need))) return CEC_EINVAL;
    for (int i = 0; i < n; ++i)
        if (u[i].src_lid >= (uint32_t)g->k || (u[i].len && !u[i].buf)) return CEC_EINVAL;
    return CEC_OK;
}

int cocytus_try_update_units_gf(cocytus_rglue *g, struct recovery *r, char *const *touch_flags,
                                const char *sub_flags, const cec_host_update *u, int n, int *need) {
    int rc = check_window(g, r, u, n, need);
    if (rc) return rc;
    int nj = 0;
    rc = try_update_window(g, r, touch_flags, NULL, sub_flags, u, n, need, &g->tmp, &nj, &g->cap_tmp);
    if (rc < 0) return rc;
    return nj ? cec_region_multiply_batch(g->tmp, nj, g->stream) : CEC_OK;
}

/* Deferred folds outlive the diffs they read (rep_queue_flush frees e->vbuf once the xid
 * is processed, rep_queue.c:86-103): the pieces of folds [from, n_fold) are copied into
 * one buffer the glue owns until the flush.  Reserved before the commit (so an ENOMEM
 * changes nothing), filled after it. */
static int own_reserve(cocytus_rglue *g, size_t total, char **buf) {
    *buf = NULL;
    if (total == 0) return CEC_OK;
    if (grow((void **)&g->owned, &g->cap_owned, g->n_owned + 1, sizeof *g->owned)) return CEC_ENOMEM;
    *buf = malloc(total);
    return *buf ? CEC_OK : CEC_ENOMEM;
}

static void own_fill(cocytus_rglue *g, int from, char *buf) {
    if (!buf) return;
    size_t o = 0;
    for (int i = from; i < g->n_fold; ++i) {
        memcpy(buf + o, g->fold[i].src, g->fold[i].len);
        g->fold[i].src = buf + o;
        o += g->fold[i].len;
    }
    g->owned[g->n_owned++] = buf;
}

/* the bytes the folds of a window read (an upper bound: every piece of a folding unit) */
static int window_fold_bytes(const cocytus_rglue *g, struct recovery *r, const char *sub_flags,
                             const cec_host_update *u, int n, size_t *total) {
    *total = 0;
    for (int i = 0; i < n; ++i) {
        const int f = try_update_walk(g, r, NULL, sub_flags, (int)u[i].src_lid, u[i].addr, (const char *)u[i].buf,
                                      u[i].len, 0, NULL, NULL);
        if (f < 0) return f;
        if (f) *total += u[i].len;
    }
    return CEC_OK;
}

static int try_update_defer(cocytus_rglue *g, struct recovery *r, char *const *touch_flags, char *touch_one,
                            const char *sub_flags, const cec_host_update *u, int n, int *need) {
    size_t total;
    int rc = window_fold_bytes(g, r, sub_flags, u, n, &total);
    if (rc) return rc;
    char *buf;
    if ((rc = own_reserve(g, total, &buf))) return rc;
    const int before = g->n_fold;
    const int ret = try_update_window(g, r, touch_flags, touch_one, sub_flags, u, n, need, &g->fold, &g->n_fold,
                                      &g->cap_fold);
    if (ret < 0) { /* (the window's checks ran in window_fold_bytes: only grow's ENOMEM) */
        g->n_fold = before;
        free(buf);
        return ret;
    }
    if (g->n_fold > before) {
        own_fill(g, before, buf);
        g->req_fold++;
    } else {
        free(buf);
    }
    return ret;
}

int cocytus_try_update_units_defer(cocytus_rglue *g, struct recovery *r, char *const *touch_flags,
                                   const char *sub_flags, const cec_host_update *u, int n, int *need) {
    int rc = check_window(g, r, u, n, need);
    if (rc) return rc;
    rc = try_update_defer(g, r, touch_flags, NULL, sub_flags, u, n, need);
    return rc < 0 ? rc : CEC_OK;
}

int cocytus_try_update_unit_defer(cocytus_rglue *g, struct recovery *r, char *touch_flags, const char *sub_flags,
                                  int peerid, uint64_t addr, const char *data, uint32_t size) {
    if (!g || !r || !r->units || peerid < 0 || peerid >= g->k || (size && !data)) return CEC_EINVAL;
    const cec_host_update x = one_update(peerid, addr, data, size);
    return try_update_defer(g, r, NULL, touch_flags, sub_flags, &x, 1, NULL);
}

int cocytus_fold_hook(const cec_host_update *u, int n, int *need, void *ctx) {
    cocytus_fold_ctx *f = ctx;
    if (!f) return CEC_EINVAL;
    return f->defer ? cocytus_try_update_units_defer(f->g, f->r, f->touch_flags, f->sub_flags, u, n, need)
                    : cocytus_try_update_units_gf(f->g, f->r, f->touch_flags, f->sub_flags, u, n, need);
}

int cocytus_recovery_queued(const cocytus_rglue *g, const cec_region_job **folds, int *n_folds,
                            const cec_region_job **solves, int *n_solves) {
    if (!g) return CEC_EINVAL;
    if (folds) *folds = g->fold;
    if (n_folds) *n_folds = g->n_fold;
    if (solves) *solves = g->solve;
    if (n_solves) *n_solves = g->n_solve;
    return CEC_OK;
}

/* complete_recovery_bottom_half (memcached.c:7842-7922): the jobs of data[i] = sum_j
 * inv[i][j] * C[j], written (first term) then accumulated, appended to *jobs. */
static int build_solve(cocytus_rglue *g, struct recovery *r, const struct recovery_queue_item *it, char **data,
                       int *n_out, cec_region_job **jobs, int *nj, int *cap) {
    if (!g || !r || !r->units || !it || !data || !n_out || it->unit_begin < 0 || it->unit_end < it->unit_begin)
        return CEC_EINVAL;
    const int k = g->k, m = g->m;
    const uint32_t mask = it->mask;
    const uint64_t nbuf = (uint64_t)(it->unit_end - it->unit_begin + 1) * UNIT;
    if (nbuf > UINT32_MAX) return CEC_EINVAL;
    int lost[32], pars[32], n = 0, np = 0;
    for (int i = 0; i < k; ++i) /* :7848-7851 */
        if (!(mask & F_LID(i))) lost[n++] = i;
    for (int i = k; i < k + m; ++i) /* :7871-7886 */
        if (mask & F_LID(i)) pars[np++] = i;
    if (np != n) return CEC_EINVAL; /* :7891 assert(m == n) */
    *n_out = n;
    if (n == 0) return CEC_OK;
    int tmp[32 * 32], inv[32 * 32], nn = 0;
    for (int p = 0; p < n; ++p)
        for (int x = 0; x < n; ++x) tmp[nn++] = MAT(g, pars[p], lost[x]);
    if (jerasure_invert_matrix(tmp, inv, n, 8) != 0) return CEC_ESINGULAR; /* :7907-7908 */
    /* the sources: this parity's units (:7853-7866) or the other parities' residuals */
    for (int p = 0; p < n; ++p) {
        if (pars[p] == g->self) {
            for (int i = it->unit_begin; i <= it->unit_end; ++i)
                if (!r->units[i].data) return CEC_EINVAL;
        } else if (!it->data_from_parity || !it->data_from_parity[pars[p]]) {
            return CEC_EINVAL;
        }
    }
    const int units = it->unit_end - it->unit_begin + 1;
    int more = 0;
    for (int p = 0; p < n; ++p) more += pars[p] == g->self ? units : 1;
    int rc = grow((void **)jobs, cap, *nj + n * more, sizeof **jobs);
    if (rc) return rc;
    for (int x = 0; x < n; ++x) {
        data[x] = malloc(nbuf); /* :7911-7914 (calloc: every byte is written below) */
        if (!data[x]) {
            for (int y = 0; y < x; ++y) {
                free(data[y]);
                data[y] = NULL;
            }
            return CEC_ENOMEM;
        }
    }
    for (int x = 0; x < n; ++x)
        for (int p = 0; p < n; ++p) { /* :7916-7922, j in order: the first term writes */
            const int coef = inv[x * n + p], add = p > 0;
            if (pars[p] == g->self) {
                for (int i = it->unit_begin; i <= it->unit_end; ++i) {
                    cec_region_job *j = &(*jobs)[(*nj)++];
                    j->src = r->units[i].data;
                    j->dst = data[x] + (uint64_t)(i - it->unit_begin) * UNIT;
                    j->base = NULL;
                    j->len = UNITSIZE;
                    j->multby = coef;
                    j->add = add;
                }
            } else {
                cec_region_job *j = &(*jobs)[(*nj)++];
                j->src = it->data_from_parity[pars[p]];
                j->dst = data[x];
                j->base = NULL;
                j->len = (uint32_t)nbuf;
                j->multby = coef;
                j->add = add;
            }
        }
    return CEC_OK;
}

int cocytus_recovery_solve_gf(cocytus_rglue *g, struct recovery *r, const struct recovery_queue_item *rqit,
                              char **data, int *n_out) {
    int nj = 0;
    int rc = build_solve(g, r, rqit, data, n_out, &g->tmp, &nj, &g->cap_tmp);
    if (rc) return rc;
    if (nj && (rc = cec_region_multiply_batch(g->tmp, nj, g->stream))) {
        for (int x = 0; x < *n_out; ++x) {
            free(data[x]);
            data[x] = NULL;
        }
        return rc;
    }
    return CEC_OK;
}

int cocytus_recovery_solve_defer(cocytus_rglue *g, struct recovery *r, const struct recovery_queue_item *rqit,
                                 char **data, int *n_out) {
    if (!g) return CEC_EINVAL;
    const int rc = build_solve(g, r, rqit, data, n_out, &g->solve, &g->n_solve, &g->cap_solve);
    if (rc) return rc;
    g->req_solve++;
    return CEC_OK;
}

int cocytus_recovery_flush(cocytus_rglue *g) {
    if (!g) return CEC_EINVAL;
    const int done = g->req_fold + g->req_solve;
    if (g->n_fold) {
        const int rc = cec_region_multiply_batch(g->fold, g->n_fold, g->stream);
        if (rc) return rc;
    }
    for (int i = 0; i < g->n_owned; ++i) free(g->owned[i]);
    g->n_owned = g->n_fold = g->req_fold = 0;
    if (g->n_solve) {
        const int rc = cec_region_multiply_batch(g->solve, g->n_solve, g->stream);
        if (rc) return rc;
    }
    g->n_solve = g->req_solve = 0;
    return done;
}
