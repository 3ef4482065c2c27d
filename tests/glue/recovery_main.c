/*
 * tests/glue/recovery_main.c -- integration/cocytus_recovery.c driven over the server's own
 * recovery types: compiled against the reference's recovery.h / ecmem.h / const.h
 * (-I/root/reference; the headers are used where they lie, not copied), the way the glue is
 * built in the server tree, and linked to libcocytus_ec.so.
 *
 *   recovery_main SCRIPT HEAP OUT
 *
 * HEAP: a binary file loaded whole; the parity arena (ecmem->mem) is its first bytes, and
 * every data buffer an op names is a byte offset into it.  SCRIPT: one op per line:
 *   init K M SELF NUNITS        struct recovery with NUNITS units, touch_flags per lid
 *   sub I V                     sub_flags[I] = V (sub_flags allocated on first use)
 *   flag I V OFF                units[I].flags = V; OFF >= 0: units[I].data = copy of HEAP[OFF..+4096)
 *   R PEER UB UE OFF            cocytus_recover_units_gf(data = HEAP+OFF)
 *   D PEER UB UE OFF            cocytus_recover_units_defer(take = 0)
 *   T PEER ADDR SIZE OFF        cocytus_try_update_unit_gf
 *   t PEER ADDR SIZE OFF        cocytus_try_update_unit_defer
 *   W N / w N                   cocytus_try_update_units_gf / _defer over the next N lines
 *                               "LID ADDR SIZE OFF"
 *   S UB UE MASK O_0 .. O_{k+m-1}   cocytus_recovery_solve_gf; O_l = data_from_parity[l]
 *                               (HEAP offset, -1 = NULL); outputs appended to OUT.solves
 *   Q ...                       cocytus_recovery_solve_defer (outputs appended at the next F)
 *   F                           cocytus_recovery_flush
 *   P                           list the queued jobs (no GPU needed)
 *   V N                         cocytus_set_diffs_gf (integration/cocytus_set.c) for the next
 *                               N lines "ADDR SIZE OFF" (value = HEAP+OFF, old bytes = the arena
 *                               at ADDR); the diffs appended to OUT.solves
 *   Z LID N DEFER               a drain window during recovery: N queued diffs of data peer
 *                               LID on the next N lines "ADDR SIZE OFF" (xids 1..N), drained by
 *                               cocytus_drain_gf with the recovery fold hook (DEFER: queued
 *                               folds) into the parity arena = HEAP's first bytes, registered
 *                               with cec_host_register (the unchanged server's host ecmem)
 * OUT.log: one line per op ("R rc", "T ret", "W rc need...", "S rc n", "F rc", "J ...").
 * OUT.units: per unit u32 flags, u8 present, 4096 bytes if present; then NUNITS bytes of
 * touch_flags per lid.  OUT.solves: the solve outputs, in op order.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cocytus_ec.h>

#include "cocytus_drain.h"
#include "cocytus_recovery.h"
#include "cocytus_set.h"
#include "rep_queue.h"

#define MAXL 64

static char *heap;
static size_t heap_len;
static struct recovery rec;
static int nunits, K, M, g_self;
static char *touch[MAXL];
static char *sub_flags;

static uint32_t z_nbytes(void *item, void *ctx) {
    (void)ctx;
    return *(uint32_t *)item;
}

static uint64_t fnv(const char *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)p[i]) * 1099511628211ull;
    return h;
}

static void desc(FILE *log, const void *p, size_t len) {
    const char *c = p;
    if (!c) {
        fprintf(log, " -");
        return;
    }
    if (c >= heap && c + len <= heap + heap_len) {
        fprintf(log, " h:%llu", (unsigned long long)(c - heap));
        return;
    }
    for (int i = 0; i < nunits; ++i)
        if (rec.units[i].data && c >= rec.units[i].data && c + len <= rec.units[i].data + UNITSIZE) {
            fprintf(log, " u:%d:%llu", i, (unsigned long long)(c - rec.units[i].data));
            return;
        }
    fprintf(log, " k:%016llx", (unsigned long long)fnv(c, len)); /* a copy the glue owns: by content */
}

static void list_jobs(FILE *log, const char *what, const cec_region_job *j, int n) {
    for (int i = 0; i < n; ++i) {
        fprintf(log, "J %s", what);
        desc(log, j[i].src, j[i].len);
        desc(log, j[i].dst, j[i].len);
        desc(log, j[i].base, j[i].len);
        fprintf(log, " %u %d %d\n", j[i].len, j[i].multby, j[i].add);
    }
}

int main(int argc, char **argv) {
    if (argc != 4) return 1;
    FILE *hf = fopen(argv[2], "rb");
    if (!hf) return 1;
    fseek(hf, 0, SEEK_END);
    heap_len = (size_t)ftell(hf);
    fseek(hf, 0, SEEK_SET);
    if (posix_memalign((void **)&heap, 4096, heap_len + 4096) || fread(heap, 1, heap_len, hf) != heap_len) return 1;
    fclose(hf);
    FILE *sc = fopen(argv[1], "r");
    char path[4096];
    snprintf(path, sizeof path, "%s.log", argv[3]);
    FILE *log = fopen(path, "w");
    snprintf(path, sizeof path, "%s.solves", argv[3]);
    FILE *solves = fopen(path, "wb");
    if (!sc || !log || !solves) return 1;
    struct ecmem ecm;
    memset(&ecm, 0, sizeof ecm);
    ecm.mem = heap;
    ecm.size = heap_len;
    cocytus_rglue *g = NULL;
    int *matrix = NULL;
    char *pending_out[256][CEC_MAX_M];
    int pending_n[256], n_pending = 0;
    uint64_t pending_nbuf[256];
    char op[8];
    while (fscanf(sc, "%7s", op) == 1) {
        if (!strcmp(op, "init")) {
            int self;
            if (fscanf(sc, "%d %d %d %d", &K, &M, &self, &nunits) != 4) return 2;
            g_self = self;
            matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
            rec.units = calloc((size_t)nunits, sizeof *rec.units);
            for (int l = 0; l < K + M; ++l) touch[l] = calloc((size_t)nunits, 1);
            if (cocytus_rglue_create(&g, K, M, matrix, self, NULL)) return 2;
        } else if (!strcmp(op, "sub")) {
            int i, v;
            if (fscanf(sc, "%d %d", &i, &v) != 2) return 2;
            if (!sub_flags) sub_flags = calloc((size_t)nunits, 1);
            sub_flags[i] = (char)v;
        } else if (!strcmp(op, "flag")) {
            int i;
            unsigned long v;
            long long off;
            if (fscanf(sc, "%d %lu %lld", &i, &v, &off) != 3) return 2;
            rec.units[i].flags = (uint32_t)v;
            if (off >= 0) {
                rec.units[i].data = malloc(UNITSIZE);
                memcpy(rec.units[i].data, heap + off, UNITSIZE);
            }
        } else if (!strcmp(op, "R") || !strcmp(op, "D")) {
            int peer, ub, ue;
            long long off;
            if (fscanf(sc, "%d %d %d %lld", &peer, &ub, &ue, &off) != 4) return 2;
            const int rc = op[0] == 'R' ? cocytus_recover_units_gf(g, &rec, &ecm, peer, ub, ue, heap + off)
                                        : cocytus_recover_units_defer(g, &rec, &ecm, peer, ub, ue, heap + off, 0);
            fprintf(log, "%s %d\n", op, rc);
        } else if (!strcmp(op, "T") || !strcmp(op, "t")) {
            int peer;
            unsigned long long addr;
            unsigned size;
            long long off;
            if (fscanf(sc, "%d %llu %u %lld", &peer, &addr, &size, &off) != 4) return 2;
            const int rc = op[0] == 'T'
                               ? cocytus_try_update_unit_gf(g, &rec, touch[peer], sub_flags, peer, addr, heap + off, size)
                               : cocytus_try_update_unit_defer(g, &rec, touch[peer], sub_flags, peer, addr, heap + off,
                                                               size);
            fprintf(log, "%s %d\n", op, rc);
        } else if (!strcmp(op, "W") || !strcmp(op, "w")) {
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
            const int rc = op[0] == 'W' ? cocytus_try_update_units_gf(g, &rec, touch, sub_flags, u, n, need)
                                        : cocytus_try_update_units_defer(g, &rec, touch, sub_flags, u, n, need);
            fprintf(log, "%s %d", op, rc);
            for (int i = 0; i < n; ++i) fprintf(log, " %d", need[i]);
            fprintf(log, "\n");
            free(u);
            free(need);
        } else if (!strcmp(op, "S") || !strcmp(op, "Q")) {
            struct recovery_queue_item it;
            memset(&it, 0, sizeof it);
            unsigned long mask;
            if (fscanf(sc, "%d %d %lu", &it.unit_begin, &it.unit_end, &mask) != 3) return 2;
            it.mask = (uint32_t)mask;
            it.data_from_parity = calloc((size_t)(K + M), sizeof(char *));
            for (int l = 0; l < K + M; ++l) {
                long long off;
                if (fscanf(sc, "%lld", &off) != 1) return 2;
                it.data_from_parity[l] = off >= 0 ? heap + off : NULL;
            }
            const uint64_t nbuf = (uint64_t)(it.unit_end - it.unit_begin + 1) * UNITSIZE;
            char *data[CEC_MAX_M] = {0};
            int n = -1;
            const int rc = op[0] == 'S' ? cocytus_recovery_solve_gf(g, &rec, &it, data, &n)
                                        : cocytus_recovery_solve_defer(g, &rec, &it, data, &n);
            fprintf(log, "%s %d %d\n", op, rc, n);
            if (rc == 0 && op[0] == 'S') {
                for (int x = 0; x < n; ++x) {
                    fwrite(data[x], 1, nbuf, solves);
                    free(data[x]);
                }
            } else if (rc == 0) {
                memcpy(pending_out[n_pending], data, sizeof data);
                pending_n[n_pending] = n;
                pending_nbuf[n_pending++] = nbuf;
            }
            free(it.data_from_parity);
        } else if (!strcmp(op, "F")) {
            const int rc = cocytus_recovery_flush(g);
            fprintf(log, "F %d\n", rc);
            for (int q = 0; q < n_pending; ++q)
                for (int x = 0; x < pending_n[q]; ++x) {
                    if (rc >= 0) fwrite(pending_out[q][x], 1, pending_nbuf[q], solves);
                    free(pending_out[q][x]);
                }
            n_pending = 0;
        } else if (!strcmp(op, "Z")) {
            int lid, n, defer;
            if (fscanf(sc, "%d %d %d", &lid, &n, &defer) != 3) return 2;
            static uint8_t *alias;
            static cec_drainer *dr;
            if (!alias) {
                if (cec_host_register(heap, heap_len, &alias) ||
                    cec_drainer_create(&dr, K, M, matrix, g_self, 4 << 20)) {
                    fprintf(stderr, "Z setup: %s\n", cec_last_error());
                    return 3;
                }
            }
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
            cocytus_fold_ctx fc;
            memset(&fc, 0, sizeof fc);
            fc.g = g;
            fc.r = &rec;
            for (int l = 0; l < K + M; ++l) fc.touch_flags[l] = touch[l];
            fc.sub_flags = sub_flags;
            fc.defer = defer;
            cocytus_drain_hooks hooks = {.item_nbytes = z_nbytes, .try_update_batch = cocytus_fold_hook, .ctx = &fc};
            cec_host_update *scratch = calloc((size_t)n + 1, sizeof *scratch);
            const int rc = cocytus_drain_gf(&q, lid, 0, (uint64_t)n, &hooks, dr, alias, NULL, scratch, n);
            fprintf(log, "Z %d\n", rc);
            free(scratch);
            free(nb);
            free(q.items);
        } else if (!strcmp(op, "V")) {
            int n;
            if (fscanf(sc, "%d", &n) != 1) return 2;
            cocytus_set_diff *sd = calloc((size_t)n + 1, sizeof *sd);
            for (int i = 0; i < n; ++i) {
                unsigned long long addr;
                unsigned size;
                long long off;
                if (fscanf(sc, "%llu %u %lld", &addr, &size, &off) != 3) return 2;
                sd[i].addr = addr;
                sd[i].nbytes = size;
                sd[i].value = heap + off;
                sd[i].diff = malloc((size_t)size + 16);
            }
            const int rc = cocytus_set_diffs_gf(&ecm, sd, n, NULL);
            fprintf(log, "V %d\n", rc);
            for (int i = 0; i < n; ++i) {
                if (rc == 0) fwrite(sd[i].diff, 1, sd[i].nbytes, solves);
                free(sd[i].diff);
            }
            free(sd);
        } else if (!strcmp(op, "P")) {
            const cec_region_job *f, *s;
            int nf, ns;
            cocytus_recovery_queued(g, &f, &nf, &s, &ns);
            fprintf(log, "P %d %d %d\n", cocytus_recovery_pending(g), nf, ns);
            list_jobs(log, "fold", f, nf);
            list_jobs(log, "solve", s, ns);
        } else {
            fprintf(stderr, "unknown op %s\n", op);
            return 2;
        }
        fflush(log);
    }
    snprintf(path, sizeof path, "%s.units", argv[3]);
    FILE *uf = fopen(path, "wb");
    if (!uf) return 1;
    for (int i = 0; i < nunits; ++i) {
        const uint8_t present = rec.units[i].data != NULL;
        fwrite(&rec.units[i].flags, 4, 1, uf);
        fwrite(&present, 1, 1, uf);
        if (present) fwrite(rec.units[i].data, 1, UNITSIZE, uf);
    }
    for (int l = 0; l < K + M; ++l) fwrite(touch[l], 1, (size_t)nunits, uf);
    fwrite(heap, 1, (size_t)nunits * UNITSIZE, uf); /* the parity arena afterwards */
    fclose(uf);
    fclose(log);
    fclose(solves);
    for (int i = 0; i < nunits; ++i) free(rec.units[i].data);
    free(rec.units);
    for (int l = 0; l < K + M; ++l) free(touch[l]);
    free(sub_flags);
    cocytus_rglue_destroy(g);
    free(matrix);
    free(heap);
    return 0;
}
