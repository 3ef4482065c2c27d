/*
 * jerasure.h -- drop-in for the part of Jerasure 2.x <jerasure.h> Cocytus uses
 * (/root/reference/memcached.c:81-84, /root/reference/recovery.h:27).
 */
#ifndef COCYTUS_EC_JERASURE_H
#define COCYTUS_EC_JERASURE_H

#include "galois.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Gauss-Jordan inverse over GF(2^8) (memcached.c:7907).  inv: caller-allocated
 * rows*rows ints.  mat is clobbered.  Returns 0, or -1 if singular.  w must be 8. */
int jerasure_invert_matrix(int *mat, int *inv, int rows, int w);

/* Product of matrices over GF(2^w) (convenience; w = 8).  Returns malloc'd r1*c2. */
int *jerasure_matrix_multiply(int *m1, int *m2, int r1, int c1, int r2, int c2, int w);

#ifdef __cplusplus
}
#endif
#endif
