/*
 * tests/glue/drain_main.c -- integration/cocytus_drain.c driven over the server's own
 * queue type: compiled against the reference's rep_queue.h (-I/root/reference; the
 * header is used where it lies, not copied), the way the glue is built in the server tree.
 *
 *   drain_main collect IN OUT   host only: cocytus_drain_collect; OUT = one line per
 *                               collected update "entry addr len lid", or "rc N"
 *   drain_main apply IN OUT     GPU: cocytus_drain_gf into a device parity arena that
 *                               starts from IN's parity bytes; OUT = the arena afterwards
 *
 * IN (little-endian): int32 lid, self_lid, k, m, ring_cap, tail, n_entries, arena_bytes,
 * cap; uint64 done_xid, stable_xid; n_entries x {uint64 xid, uint64 addr, int32 len,
 * int32 vnbytes, int32 veto}; the entries' diff bytes back to back (len each); then
 * arena_bytes of initial parity.  Entry e sits at ring index tail + e.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cocytus_ec.h>
#include <reed_sol.h>

#include "cocytus_drain.h"
#include "rep_queue.h"

struct test_item { /* what item_nbytes reads: the test's own value record */
    uint32_t nbytes;
    int veto;
};

static uint32_t item_nbytes(void *item, void *ctx) {
    (void)ctx;
    return ((struct test_item *)item)->nbytes;
}

static int vetoes; /* try_update calls that kept a diff out of the arena */

static int try_update(int lid, uint64_t addr, char *buf, uint32_t nbytes, void *ctx) {
    /* the test's recovery fold: the entry's veto flag, found by its buffer */
    struct test_item *items = ctx;
    (void)lid; (void)addr; (void)nbytes;
    int veto = items[((int32_t *)buf)[-1]].veto; /* entry index stored before the bytes */
    vetoes += veto;
    return !veto;
}

static void rd(FILE *f, void *p, size_t n) {
    if (n && fread(p, 1, n, f) != n) {
        fprintf(stderr, "short input\n");
        exit(3);
    }
}

int main(int argc, char **argv) {
    if (argc != 4) return 1;
    const int apply = !strcmp(argv[1], "apply");
    FILE *in = fopen(argv[2], "rb");
    if (!in) return 1;
    int32_t h[9];
    uint64_t x[2];
    rd(in, h, sizeof h);
    rd(in, x, sizeof x);
    const int lid = h[0], self = h[1], K = h[2], M = h[3], ring = h[4], tail = h[5], n = h[6];
    const size_t arena = (size_t)(uint32_t)h[7];
    const int cap = h[8];
    struct rep_queue q;
    q.cap = (uint32_t)ring;
    q.items = calloc((size_t)ring, sizeof(struct rep_queue_item));
    q.tail = (uint32_t)tail;
    q.head = (uint32_t)(tail + n);
    struct test_item *items = calloc((size_t)n + 1, sizeof *items);
    int64_t *idx_of = calloc((size_t)n + 1, sizeof *idx_of);
    for (int e = 0; e < n; ++e) {
        uint64_t xa[2];
        int32_t li[3];
        rd(in, xa, sizeof xa);
        rd(in, li, sizeof li);
        struct rep_queue_item *it = &q.items[(uint32_t)(tail + e) % q.cap];
        memset(it, 0, sizeof *it);
        it->xid = xa[0];
        it->lid = lid;
        it->addr = xa[1];
        it->vnbytes = li[1];
        it->item = &items[e];
        items[e].nbytes = (uint32_t)li[0];
        items[e].veto = li[2];
    }
    for (int e = 0; e < n; ++e) { /* each diff in its own malloc'd vbuf, as conn_nread leaves it */
        struct rep_queue_item *it = &q.items[(uint32_t)(tail + e) % q.cap];
        int32_t *blk = malloc(sizeof(int32_t) + (size_t)it->vnbytes + 1);
        blk[0] = e;
        it->vbuf = (char *)(blk + 1);
        rd(in, it->vbuf, items[e].nbytes);
    }
    cocytus_drain_hooks hooks = {item_nbytes, try_update, items};
    cec_host_update *scratch = calloc((size_t)cap + 1, sizeof *scratch);
    FILE *out = fopen(argv[3], apply ? "wb" : "w");
    if (!out) return 1;
    if (!apply) {
        const int rc = cocytus_drain_collect(&q, lid, x[0], x[1], &hooks, scratch, cap);
        if (rc < 0) {
            fprintf(out, "rc %d\n", rc);
        } else {
            for (int i = 0; i < rc; ++i) {
                const int e = ((const int32_t *)scratch[i].buf)[-1];
                fprintf(out, "%d %llu %u %u\n", e, (unsigned long long)scratch[i].addr, scratch[i].len,
                        scratch[i].src_lid);
            }
        }
        fclose(out);
        return 0;
    }
    uint8_t *host = malloc(arena);
    rd(in, host, arena);
    fclose(in);
    if (cec_device_check() != CEC_OK) {
        fprintf(stderr, "%s\n", cec_last_error());
        return 2;
    }
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8);
    uint8_t *parity;
    void *slab;
    cec_drainer *dr;
    if (cec_arenas_alloc(1, arena, &parity, &slab) || cec_copy(parity, host, arena, NULL) ||
        cec_stream_synchronize(NULL) || cec_drainer_create(&dr, K, M, matrix, self, 1 << 20)) {
        fprintf(stderr, "setup: %s\n", cec_last_error());
        return 2;
    }
    const int applied = cocytus_drain_gf(&q, lid, x[0], x[1], &hooks, dr, parity, NULL, scratch, cap);
    if (applied < 0) {
        fprintf(stderr, "cocytus_drain_gf: %d %s\n", applied, cec_last_error());
        return 2;
    }
    if (cec_copy(host, parity, arena, NULL) || cec_stream_synchronize(NULL)) return 2;
    fwrite(host, 1, arena, out);
    fclose(out);
    printf("applied %d vetoed %d launches %d\n", applied, vetoes, cec_drainer_last_launches(dr));
    cec_drainer_destroy(dr);
    cec_arenas_free(slab);
    free(matrix);
    return 0;
}
