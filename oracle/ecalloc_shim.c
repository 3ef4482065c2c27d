/* oracle/ecalloc_shim.c -- TEST INFRASTRUCTURE.  A flat C entry point around the
 * reference's own arena allocator, compiled together with the unmodified sources
 * /root/reference/ecalloc.c and /root/reference/avltree.c into oracle/_ref/ (see
 * oracle/Makefile `ref`).  It lets the tests take value addresses from the real
 * allocator (ecalloc.c:168-229, 16-B rounding at :176) instead of
 * a restatement of it.  struct ecalloc's layout stays private to this file. */
#include <stdint.h>
#include <stdlib.h>

#include "ecalloc.h"

void *ref_ecalloc_create(uint64_t size) {
    struct ecalloc *a = malloc(sizeof *a);
    if (a) ecalloc_init(a, size);
    return a;
}

uint64_t ref_ec_alloc(void *a, uint64_t size) { return ec_alloc((struct ecalloc *)a, size); }

void ref_ec_free(void *a, uint64_t addr) { ec_free((struct ecalloc *)a, addr); }

uint64_t ref_ec_used(void *a) { return ((struct ecalloc *)a)->used; }
