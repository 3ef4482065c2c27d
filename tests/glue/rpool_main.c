/*
 * tests/glue/rpool_main.c -- integration/cocytus_recovery_pool.c driven over the server's own
 * recovery types (the reference's recovery.h / ecmem.h / const.h / rep_queue.h used where
 * they lie, -I/root/reference), linked to libcocytus_ec.so.  Needs a GPU (the pool's
 * residual is in HBM).
 *
 *   rpool_main SCRIPT HEAP OUT
 *
 * HEAP: a binary file loaded whole; the parity arena is its first NUNITS x 4096 bytes,
 * registered with cec_host_register (the unchanged server's host ecmem: the pool reads the
 * first-touch parity units in place, the drain applies into it); every data buffer an op
 * names is a byte offset into HEAP.  SCRIPT: one op per line:
 *   init K M SELF NUNITS QCAP CAP   struct recovery (NUNITS units, a QCAP-item queue),
 *                                   cocytus_rpool_create with CAP residual units
 *   sub I V                         sub_flags[I] = V
 *   flag I V                        units[I].flags = V
 *   B QI UB UE MASK                 queue.items[QI] = request [UB, UE] of MASK; cocytus_rpool_begin
 *   b QI                            cocytus_rpool_begin of queue.items[QI] again, unchanged
 *   E QI                            cocytus_rpool_end, then recovery_req_remove's reset
 *                                   (recovery.c:190-211: the units' flags = 0)
 *   R QI PEER OFF / r QI PEER OFF   cocytus_rpool_recover_units (r: received into
 *                                   cocytus_rpool_staging first)
 *   T PEER ADDR SIZE OFF            cocytus_rpool_try_update_unit
 *   W N                             cocytus_rpool_try_update_units over the next N lines
 *                                   "LID ADDR SIZE OFF"
 *   Z LID N                         a drain window (N diffs of LID on the next N lines
 *                                   "ADDR SIZE OFF", xids 1..N) through cocytus_drain_gf with
 *                                   cocytus_rpool_fold_hook, applied into the arena
 *   S QI O_0 .. O_{k+m-1}           cocytus_rpool_solve (O_l = data_from_parity[l], -1 NULL)
 *   F                               cocytus_rpool_flush; then data[0..n) of every request
 *                                   solved by it, in S order, appended to OUT.solves
 *   X QI                            cocytus_rpool_residual appended to OUT.solves
 * OUT.log: one line per op; OUT.units: u32 flags per unit, NUNITS bytes of touch_flags per
 * lid, the arena afterwards.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cocytus_ec.h>

#include "cocytus_drain.h"
#include "cocytus_recovery_pool.h"
#include "rep_queue.h"

#define MAXL 64

static uint32_t z_nbytes(void *item, void *ctx) {
    (void)ctx;
    return *(uint32_t *)item;
}

int main(int argc, char **argv) {
    if (argc != 4) return 1;
    FILE *hf = fopen(argv[2], "rb");
    if (!hf) return 1;
    fseek(hf, 0, SEEK_END);
    const size_t heap_len = (size_t)ftell(hf);
    fseek(hf, 0, SEEK_SET);
    char *heap;
    if (posix_memalign((void **)&heap, 4096, heap_len + 4096) || fread(heap, 1, heap_len, hf) != heap_len) return 1;
    fclose(hf);
    FILE *sc = fopen(argv[1], "r");
    char path[4096];
    snprintf(path, sizeof path, "%s.log", argv[3]);
    FILE *log = fopen(path, "w");
    snprintf(path, sizeof path, "%s.solves", argv[3]);
    FILE *solves = fopen(path, "wb");
    if (!sc || !log || !solves) return 1;
    struct recovery rec;
    memset(&rec, 0, sizeof rec);
    cocytus_rpool *g = NULL;
    cec_drainer *dr = NULL;
    int *matrix = NULL, K = 0, M = 0, self = 0, nunits = 0, qcap = 0;
    char *touch[MAXL] = {0}, *sub_flags = NULL;
    uint8_t *alias = NULL;
    int *solved = NULL, n_solved = 0;
    char op[8];
    while (fscanf(sc, "%7s", op) == 1) {
        if (!strcmp(op, "init")) {
            int cap;
            if (fscanf(sc, "%d %d %d %d %d %d", &K, &M, &self, &nunits, &qcap, &cap) != 6) return 2;
            matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
            rec.units = calloc((size_t)nunits, sizeof *rec.units);
            rec.queue.cap = qcap;
            rec.queue.items = calloc((size_t)qcap, sizeof *rec.queue.items);
            solved = calloc((size_t)qcap * 4 + 1, sizeof *solved);
            for (int l = 0; l < K + M; ++l) touch[l] = calloc((size_t)nunits, 1);
            if (cec_host_register(heap, (size_t)nunits * UNITSIZE, &alias) ||
                cocytus_rpool_create(&g, K, M, matrix, self, alias, qcap, cap, NULL) ||
                cec_drainer_create(&dr, K, M, matrix, self, 4 << 20)) {
                fprintf(stderr, "init: %s\n", cec_last_error());
                return 3;
            }
        } else if (!strcmp(op, "sub")) {
            int i, v;
            if (fscanf(sc, "%d %d", &i, &v) != 2) return 2;
            if (!sub_flags) sub_flags = calloc((size_t)nunits, 1);
            sub_flags[i] = (char)v;
        } else if (!strcmp(op, "flag")) {
            int i;
            unsigned long v;
            if (fscanf(sc, "%d %lu", &i, &v) != 2) return 2;
            rec.units[i].flags = (uint32_t)v;
        } else if (!strcmp(op, "B")) {
            int qi, ub, ue;
            unsigned long mask;
            if (fscanf(sc, "%d %d %d %lu", &qi, &ub, &ue, &mask) != 4) return 2;
            struct recovery_queue_item *it = &rec.queue.items[qi];
            free(it->data_from_parity);
            memset(it, 0, sizeof *it);
            it->unit_begin = ub;
            it->unit_end = ue;
            it->mask = (uint32_t)mask;
            it->in_use = 1;
            it->data_from_parity = calloc((size_t)(K + M), sizeof(char *));
            fprintf(log, "B %d\n", cocytus_rpool_begin(g, &rec, it));
        } else if (!strcmp(op, "b")) { /* the same request begun again */
            int qi;
            if (fscanf(sc, "%d", &qi) != 1) return 2;
            fprintf(log, "b %d\n", cocytus_rpool_begin(g, &rec, &rec.queue.items[qi]));
        } else if (!strcmp(op, "E")) {
            int qi;
            if (fscanf(sc, "%d", &qi) != 1) return 2;
            struct recovery_queue_item *it = &rec.queue.items[qi];
            fprintf(log, "E %d\n", cocytus_rpool_end(g, &rec, it));
            for (int i = it->unit_begin; i <= it->unit_end; ++i) rec.units[i].flags = 0; /* recovery.c:200-205 */
            it->in_use = 0;
        } else if (!strcmp(op, "R") || !strcmp(op, "r")) {
            int qi, peer;
            long long off;
            if (fscanf(sc, "%d %d %lld", &qi, &peer, &off) != 3) return 2;
            const struct recovery_queue_item *it = &rec.queue.items[qi];
            const char *data = heap + off;
            if (op[0] == 'r') { /* received in place (c->ritem = the staging) */
                char *st = cocytus_rpool_staging(g, &rec, it, peer);
                if (st) {
                    memcpy(st, data, (size_t)(it->unit_end - it->unit_begin + 1) * UNITSIZE);
                    data = st;
                }
            }
            fprintf(log, "%s %d\n", op, cocytus_rpool_recover_units(g, &rec, it, peer, data));
        } else if (!strcmp(op, "T")) {
            int peer;
            unsigned long long addr;
            unsigned size;
            long long off;
            if (fscanf(sc, "%d %llu %u %lld", &peer, &addr, &size, &off) != 4) return 2;
            fprintf(log, "T %d\n", cocytus_rpool_try_update_unit(g, &rec, touch[peer], sub_flags, peer, addr,
                                                                 heap + off, size));
        } else if (!strcmp(op, "W")) {
            int n;
            if (fscanf(sc, "%d", &n) != 1) return 2;
            cec_host_update *u = calloc((size_t)n + 1, sizeof *u);
            int *need = calloc((size_t)n + 1, sizeof *need);
            for (int i = 0; i < n; ++i) {
                int lid;
                unsigned long long addr;
                unsigned size;
                long long off;
                if (fscanf(sc, "%d %llu %u %lld", &lid, &addr, &size, &off) != 4) return 2;
                u[i].buf = heap + off;
                u[i].addr = addr;
                u[i].len = size;
                u[i].src_lid = (uint32_t)lid;
            }
            const int rc = cocytus_rpool_try_update_units(g, &rec, touch, sub_flags, u, n, need);
            fprintf(log, "W %d", rc);
            for (int i = 0; i < n; ++i) fprintf(log, " %d", need[i]);
            fprintf(log, "\n");
            free(u);
            free(need);
        } else if (!strcmp(op, "Z")) {
            int lid, n;
            if (fscanf(sc, "%d %d", &lid, &n) != 2) return 2;
            struct rep_queue q;
            q.cap = (uint32_t)n + 1;
            q.items = calloc((size_t)n + 1, sizeof *q.items);
            q.tail = 0;
            q.head = (uint32_t)n;
            uint32_t *nb = calloc((size_t)n + 1, sizeof *nb);
            for (int i = 0; i < n; ++i) {
                unsigned long long addr;
                long long off;
                if (fscanf(sc, "%llu %u %lld", &addr, &nb[i], &off) != 3) return 2;
                q.items[i].xid = (uint64_t)i + 1;
                q.items[i].lid = lid;
                q.items[i].addr = addr;
                q.items[i].vbuf = heap + off;
                q.items[i].vnbytes = (int)nb[i];
                q.items[i].item = &nb[i];
            }
            cocytus_rpool_fold_ctx fc;
            memset(&fc, 0, sizeof fc);
            fc.g = g;
            fc.r = &rec;
            for (int l = 0; l < K + M; ++l) fc.touch_flags[l] = touch[l];
            fc.sub_flags = sub_flags;
            cocytus_drain_hooks hooks = {.item_nbytes = z_nbytes, .try_update_batch = cocytus_rpool_fold_hook,
                                         .ctx = &fc};
            cec_host_update *scratch = calloc((size_t)n + 1, sizeof *scratch);
            fprintf(log, "Z %d\n", cocytus_drain_gf(&q, lid, 0, (uint64_t)n, &hooks, dr, alias, NULL, scratch, n));
            free(scratch);
            free(nb);
            free(q.items);
        } else if (!strcmp(op, "S")) {
            int qi;
            if (fscanf(sc, "%d", &qi) != 1) return 2;
            struct recovery_queue_item *it = &rec.queue.items[qi];
            for (int l = 0; l < K + M; ++l) {
                long long off;
                if (fscanf(sc, "%lld", &off) != 1) return 2;
                it->data_from_parity[l] = off >= 0 ? heap + off : NULL;
            }
            int n = -1;
            const int rc = cocytus_rpool_solve(g, &rec, it, &n);
            fprintf(log, "S %d %d\n", rc, n);
            if (rc == 0 && n > 0) {
                if (n_solved == qcap * 4) return fprintf(stderr, "more than %d solves between flushes\n", qcap * 4), 2;
                solved[n_solved++] = qi;
            }
        } else if (!strcmp(op, "F")) {
            const int rc = cocytus_rpool_flush(g);
            fprintf(log, "F %d\n", rc);
            for (int s = 0; s < n_solved && rc >= 0; ++s) {
                const struct recovery_queue_item *it = &rec.queue.items[solved[s]];
                const size_t nbuf = (size_t)(it->unit_end - it->unit_begin + 1) * UNITSIZE;
                for (int x = 0;; ++x) {
                    const char *d = cocytus_rpool_data(g, &rec, it, x);
                    if (!d) break;
                    fwrite(d, 1, nbuf, solves);
                }
            }
            n_solved = 0;
        } else if (!strcmp(op, "X")) {
            int qi;
            if (fscanf(sc, "%d", &qi) != 1) return 2;
            const struct recovery_queue_item *it = &rec.queue.items[qi];
            const size_t nbuf = (size_t)(it->unit_end - it->unit_begin + 1) * UNITSIZE;
            char *buf = malloc(nbuf);
            const int rc = cocytus_rpool_residual(g, &rec, it, buf);
            fprintf(log, "X %d\n", rc);
            if (rc == 0) fwrite(buf, 1, nbuf, solves);
            free(buf);
        } else {
            fprintf(stderr, "unknown op %s\n", op);
            return 2;
        }
        fflush(log);
    }
    snprintf(path, sizeof path, "%s.units", argv[3]);
    FILE *uf = fopen(path, "wb");
    if (!uf) return 1;
    for (int i = 0; i < nunits; ++i) fwrite(&rec.units[i].flags, 4, 1, uf);
    for (int l = 0; l < K + M; ++l) fwrite(touch[l], 1, (size_t)nunits, uf);
    fwrite(heap, 1, (size_t)nunits * UNITSIZE, uf);
    fclose(uf);
    fclose(log);
    fclose(solves);
    fprintf(stderr, "teardown: pool\n");
    cocytus_rpool_destroy(g);
    fprintf(stderr, "teardown: drainer\n");
    cec_drainer_destroy(dr);
    fprintf(stderr, "teardown: unregister\n");
    cec_host_unregister(heap);
    fprintf(stderr, "teardown: free\n");
    for (int q = 0; q < qcap; ++q) free(rec.queue.items[q].data_from_parity);
    free(rec.queue.items);
    free(rec.units);
    for (int l = 0; l < K + M; ++l) free(touch[l]);
    free(sub_flags);
    free(solved);
    free(matrix);
    free(heap);
    fprintf(stderr, "teardown: exit\n");
    return 0;
}
