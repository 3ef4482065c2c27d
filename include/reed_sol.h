/*
 * reed_sol.h -- drop-in for the part of Jerasure 2.x <reed_sol.h> Cocytus uses
 * (/root/reference/memcached.c:81-84, /root/reference/recovery.h:28).
 */
#ifndef COCYTUS_EC_REED_SOL_H
#define COCYTUS_EC_REED_SOL_H

#include "jerasure.h"

#ifdef __cplusplus
extern "C" {
#endif

/* (rows x cols) systematic "big Vandermonde" distribution matrix over GF(2^8):
 * identity on top, row `cols` all ones, column 0 all ones.  Called as
 * (K+M, K, 8) at memcached.c:6845.  malloc'd (caller frees), row-major;
 * NULL if cols >= rows, rows > 256, or w != 8. */
int *reed_sol_big_vandermonde_distribution_matrix(int rows, int cols, int w);

/* The extended Vandermonde matrix it is derived from (rows x cols, malloc'd). */
int *reed_sol_extended_vandermonde_matrix(int rows, int cols, int w);

#ifdef __cplusplus
}
#endif
#endif
