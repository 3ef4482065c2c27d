/*
 * integration/cocytus_set.h -- server-side glue, data side: the SET diff of a data process
 * batched onto libcocytus_ec.
 *
 * Per SET a data process computes diff = new value ^ the bytes at the value's freshly
 * allocated arena address and ships it to every parity (complete_nread,
 * /root/reference/memcached.c:2664-2681; the substitute's twin in
 * conn_recovery_complete_for_set, :5597-5611):
 *     memcpy(diff, c->vbuf, it->nbytes);
 *     galois_w08_region_multiply(ecmem_get(&ecmem, addr), 1, it->nbytes, diff, 1);
 * one synchronous drop-in call per SET.  cocytus_set_diffs_gf computes the diffs of a whole
 * list of SETs (the SETs one event-loop pass completed) in one cec_region_multiply_batch.
 * Like the other glue, this file belongs in the server tree and uses the server's own
 * ecmem.h unchanged.
 */
#ifndef COCYTUS_SET_H
#define COCYTUS_SET_H

#include <stdint.h>

#include <cocytus_ec.h>

#include "ecmem.h" /* the server's */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cocytus_set_diff {
    const char *value; /* c->vbuf: the new value (it->nbytes bytes, CRLF included) */
    uint64_t addr;     /* it->addr, from ecmem_alloc: the old bytes are ecmem_get(ecm, addr) */
    uint32_t nbytes;   /* it->nbytes */
    char *diff;        /* out: nbytes bytes (the reference's 16-aligned malloc'd diff) */
} cocytus_set_diff;

/* diff = ecmem[addr .. addr+nbytes) ^ value for every SET, in one batch (synchronous).
 * The arena is host memory (the server's ecmem; registered or not).  Returns CEC_OK or a
 * negative cec_status (CEC_EOVERLAP: a diff buffer overlaps a value or the arena). */
int cocytus_set_diffs_gf(struct ecmem *ecm, const cocytus_set_diff *sets, int n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* COCYTUS_SET_H */
