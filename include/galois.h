/*
 * galois.h -- drop-in for Jerasure 2.x <galois.h> as used by Cocytus
 * (/root/reference/memcached.c:81-84, /root/reference/recovery.h:29), served by
 * libcocytus_ec.so (link it as -lJerasure through the libJerasure.so symlink, or
 * -lcocytus_ec).
 *
 * galois_w08_region_multiply replaces the GF-Complete region multiply behind
 * memcached.c:2681, 5611, 7764, 7918 and recovery.c:91, 123.  It runs the HIP
 * kernel on the GPU: device pointers (hipMalloc / hipHostMalloc / registered) are
 * used in place; pageable host buffers up to 256 KiB go through mapped pinned
 * staging that the kernel reads and writes over PCIe, larger ones are staged through
 * device memory.  The call is synchronous (the result is visible on return, in host
 * memory too: the kernel's waves release it at system scope before the completion
 * signal), re-entrant, and
 * accepts any alignment and any nbytes >= 0.  Like the original it has no error channel: misuse or a HIP
 * failure prints a message and aborts (there is no CPU fallback).
 */
#ifndef COCYTUS_EC_GALOIS_H
#define COCYTUS_EC_GALOIS_H

#ifdef __cplusplus
extern "C" {
#endif

/* r2 != NULL, add != 0: r2[i] ^= multby * region[i]   (every Cocytus call site)
 * r2 != NULL, add == 0: r2[i]  = multby * region[i]
 * r2 == NULL          : region[i] = multby * region[i]
 * multby in [0, 255]. */
void galois_w08_region_multiply(char *region, int multby, int nbytes, char *r2, int add);

/* Scalar GF(2^w) helpers of the same header (w = 8 only; other w abort). */
int galois_single_multiply(int a, int b, int w);
int galois_single_divide(int a, int b, int w);
int galois_inverse(int x, int w);

#ifdef __cplusplus
}
#endif
#endif
