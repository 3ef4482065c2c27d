/*
 * oracle/gf8_ref.c -- CPU restatement of the Cocytus erasure-coding hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gf8_ref.h).  PARITY UNPINNED: Jerasure 2.x /
 * GF-Complete are not in /root/reference nor in this image; the reference has
 * no EC test vectors.  Each function names the reference call site whose
 * semantics it restates.
 */
#include "gf8_ref.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define GF_POLY 0x11D /* x^8+x^4+x^3+x^2+1: Jerasure prim_poly[8] = 0435 (octal) */

static uint8_t g_exp[512];
static int g_log[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* Jerasure/GF-Complete initialise the w=8 field lazily on first use
 * (galois_init(8)); the restatement does the same, thread-safely. */
static void gf_build_tables(void)
{
    int x = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = (uint8_t)x;
        g_exp[i + 255] = (uint8_t)x;
        g_log[x] = i;
        x <<= 1;
        if (x & 0x100) x ^= GF_POLY;
    }
    g_exp[510] = g_exp[0];
    g_exp[511] = g_exp[1];
    g_log[0] = -1;
}

static void gf_init(void) { pthread_once(&g_once, gf_build_tables); }

int ref_gf_exp(int i) { gf_init(); return g_exp[((i % 255) + 255) % 255]; }
int ref_gf_log(int a) { gf_init(); return (a > 0 && a < 256) ? g_log[a] : -1; }

int ref_gf_mul(int a, int b)
{
    gf_init();
    a &= 0xFF;
    b &= 0xFF;
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

int ref_gf_div(int a, int b)
{
    gf_init();
    a &= 0xFF;
    b &= 0xFF;
    if (b == 0) return -1;
    if (a == 0) return 0;
    return g_exp[g_log[a] + 255 - g_log[b]];
}

/* galois_w08_region_multiply (Jerasure galois.c, w=8 → GF-Complete
 * multiply_region.w32 with xor = add).  Call sites: memcached.c:2681, 5611,
 * 7764, 7918; recovery.c:91, 123; microbenchmarks/galois_tp.c:42. */
void ref_region_multiply(uint8_t *region, int multby, long nbytes, uint8_t *r2, int add)
{
    gf_init();
    uint8_t tab[256];
    for (int x = 0; x < 256; ++x) tab[x] = (uint8_t)ref_gf_mul(multby, x);
    if (r2 == NULL) {
        for (long i = 0; i < nbytes; ++i) region[i] = tab[region[i]];
    } else if (add) {
        for (long i = 0; i < nbytes; ++i) r2[i] ^= tab[region[i]];
    } else {
        for (long i = 0; i < nbytes; ++i) r2[i] = tab[region[i]];
    }
}

/* Jerasure reed_sol_extended_vandermonde_matrix(rows, cols, 8): row 0 = e_0,
 * row rows-1 = e_{cols-1}, row i (0 < i < rows-1) = [i^0, i^1, ..., i^{cols-1}]. */
int *ref_extended_vandermonde(int rows, int cols)
{
    if (rows < 1 || cols < 1 || rows > 256 || cols > 256) return NULL;
    int *v = (int *)calloc((size_t)rows * cols, sizeof(int));
    if (!v) return NULL;
    v[0] = 1;
    if (rows == 1) return v;
    v[(rows - 1) * cols + (cols - 1)] = 1;
    for (int i = 1; i < rows - 1; ++i) {
        int p = 1;
        for (int j = 0; j < cols; ++j) {
            v[i * cols + j] = p;
            p = ref_gf_mul(p, i);
        }
    }
    return v;
}

/* Jerasure reed_sol_big_vandermonde_distribution_matrix(rows, cols, 8), called
 * as (K+M, K, 8) at memcached.c:6845.  Column operations turn the top cols x cols
 * block into the identity (pivot row swap, column scale, column elimination),
 * then the parity columns are scaled so row `cols` is all ones, then each later
 * parity row is scaled so its first entry is one. */
int *ref_big_vandermonde(int rows, int cols)
{
    if (cols >= rows) return NULL;
    int *d = ref_extended_vandermonde(rows, cols);
    if (!d) return NULL;
#define D(r, c) d[(r) * cols + (c)]
    for (int i = 1; i < cols; ++i) {
        int r = i;
        while (r < rows && D(r, i) == 0) ++r;
        if (r >= rows) { free(d); return NULL; }
        if (r != i) {
            for (int c = 0; c < cols; ++c) { int t = D(r, c); D(r, c) = D(i, c); D(i, c) = t; }
        }
        if (D(i, i) != 1) {
            int s = ref_gf_div(1, D(i, i));
            for (int q = 0; q < rows; ++q) D(q, i) = ref_gf_mul(s, D(q, i));
        }
        for (int c = 0; c < cols; ++c) {
            int e = D(i, c);
            if (c == i || e == 0) continue;
            for (int q = 0; q < rows; ++q) D(q, c) ^= ref_gf_mul(e, D(q, i));
        }
    }
    for (int c = 0; c < cols; ++c) {          /* row `cols` := all ones */
        int e = D(cols, c);
        if (e == 1) continue;
        int s = ref_gf_div(1, e);
        for (int q = cols; q < rows; ++q) D(q, c) = ref_gf_mul(s, D(q, c));
    }
    for (int q = cols + 1; q < rows; ++q) {   /* column 0 := all ones */
        int e = D(q, 0);
        if (e == 1) continue;
        int s = ref_gf_div(1, e);
        for (int c = 0; c < cols; ++c) D(q, c) = ref_gf_mul(D(q, c), s);
    }
#undef D
    return d;
}

/* Jerasure jerasure_invert_matrix(mat, inv, rows, 8) (memcached.c:7907):
 * forward elimination to unit upper-triangular with row swaps, then back
 * substitution.  mat is clobbered; -1 if singular. */
int ref_invert_matrix(int *mat, int *inv, int rows)
{
    const int n = rows;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) inv[i * n + j] = (i == j);
    for (int i = 0; i < n; ++i) {
        if (mat[i * n + i] == 0) {
            int r = i + 1;
            while (r < n && mat[r * n + i] == 0) ++r;
            if (r == n) return -1;
            for (int c = 0; c < n; ++c) {
                int t = mat[i * n + c]; mat[i * n + c] = mat[r * n + c]; mat[r * n + c] = t;
                t = inv[i * n + c]; inv[i * n + c] = inv[r * n + c]; inv[r * n + c] = t;
            }
        }
        int piv = mat[i * n + i];
        if (piv != 1) {
            int s = ref_gf_div(1, piv);
            for (int c = 0; c < n; ++c) {
                mat[i * n + c] = ref_gf_mul(mat[i * n + c], s);
                inv[i * n + c] = ref_gf_mul(inv[i * n + c], s);
            }
        }
        for (int r = i + 1; r < n; ++r) {
            int e = mat[r * n + i];
            if (e == 0) continue;
            for (int c = 0; c < n; ++c) {
                mat[r * n + c] ^= ref_gf_mul(e, mat[i * n + c]);
                inv[r * n + c] ^= ref_gf_mul(e, inv[i * n + c]);
            }
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        for (int r = 0; r < i; ++r) {
            int e = mat[r * n + i];
            if (e == 0) continue;
            mat[r * n + i] = 0;
            for (int c = 0; c < n; ++c) inv[r * n + c] ^= ref_gf_mul(e, inv[i * n + c]);
        }
    }
    return 0;
}

/* memcached.c:2673-2681: memcpy(diff, vbuf, n); region_multiply(old, 1, n, diff, 1) */
void ref_set_diff(const uint8_t *oldv, const uint8_t *newv, long n, uint8_t *diff)
{
    memcpy(diff, newv, (size_t)n);
    ref_region_multiply((uint8_t *)oldv, 1, n, diff, 1);
}

/* memcached.c:7762-7767 */
void ref_parity_apply(const int *matrix, int k, int lid_self, int lid_src,
                      const uint8_t *diff, long n, uint8_t *parity)
{
    ref_region_multiply((uint8_t *)diff, matrix[lid_self * k + lid_src], n, parity, 1);
}

/* complete_nread (memcached.c:2664-2700) → parity_send → process_rep_command on
 * each live parity (memcached.c:7739-7767) → conn_waiting_ack installs the new
 * value (memcached.c:5666). */
void ref_diff_update(const int *matrix, int k, int m, int shard_j,
                     uint8_t *old_in_arena, const uint8_t *newv, long n,
                     uint8_t *const *parity, int install)
{
    uint8_t *diff = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
    ref_set_diff(old_in_arena, newv, n, diff);
    for (int p = 0; p < m; ++p)
        ref_parity_apply(matrix, k, k + p, shard_j, diff, n, parity[p]);
    if (install) memcpy(old_in_arena, newv, (size_t)n);
    free(diff);
}

void ref_encode(const int *matrix, int k, int m, const uint8_t *const *data,
                uint8_t *const *parity, long n)
{
    for (int p = 0; p < m; ++p) memset(parity[p], 0, (size_t)n);
    for (int j = 0; j < k; ++j)               /* one SET per data shard, old = 0 */
        for (int p = 0; p < m; ++p)
            ref_parity_apply(matrix, k, k + p, j, data[j], n, parity[p]);
}

/* memcached.c:8136-8151 */
uint32_t ref_recovery_mask(int k, int m, int leader_lid, const int *connected)
{
    int remaining = k - 1;
    uint32_t mask = 1u << leader_lid;
    for (int i = 0; i < k + m && remaining; ++i) {
        if (i == leader_lid || !connected[i]) continue;
        mask |= 1u << i;
        --remaining;
    }
    return remaining ? 0 : mask;
}

/* recovery.c:72-94 for one range */
void ref_recover_units(const int *matrix, int k, int lid_self, int peer_lid,
                       const uint8_t *own_parity, const uint8_t *peer_data, long n,
                       uint8_t *residual, int *touched)
{
    if (!*touched) {                       /* first touch: copy parity unit, :79-82 */
        memcpy(residual, own_parity, (size_t)n);
        *touched = 1;
    }
    ref_region_multiply((uint8_t *)peer_data, matrix[lid_self * k + peer_lid], n, residual, 1);
}

/* recovery.c:123-125 */
void ref_try_update_unit(const int *matrix, int k, int lid_self, int peer_lid,
                         const uint8_t *diff, long len, uint8_t *residual_at_offset)
{
    ref_region_multiply((uint8_t *)diff, matrix[lid_self * k + peer_lid], len,
                        residual_at_offset, 1);
}

/* memcached.c:7842-7922 */
int ref_bottom_half(const int *matrix, int k, int m, uint32_t mask,
                    const uint8_t *const *C, long nbuf, uint8_t *const *out)
{
    int n = 0;
    for (int i = 0; i < k; ++i)
        if (!(mask & (1u << i))) ++n;
    if (n == 0) return 0;
    int *tmp = (int *)malloc(sizeof(int) * n * n);
    int *inv = (int *)malloc(sizeof(int) * n * n);
    int nn = 0, rows = 0;
    for (int i = k; i < k + m; ++i) {
        if (!(mask & (1u << i))) continue;
        ++rows;
        for (int j = 0; j < k; ++j)
            if (!(mask & (1u << j))) tmp[nn++] = matrix[i * k + j];
    }
    if (nn != n * n || rows != n || ref_invert_matrix(tmp, inv, n) != 0) {
        free(tmp); free(inv);
        return -1;
    }
    for (int i = 0; i < n; ++i) {
        memset(out[i], 0, (size_t)nbuf);               /* calloc, :7913 */
        for (int j = 0; j < n; ++j)
            ref_region_multiply((uint8_t *)C[j], inv[i * n + j], nbuf, out[i], 1);
    }
    free(tmp); free(inv);
    return n;
}

int ref_decode(const int *matrix, int k, int m, uint32_t mask,
               const uint8_t *const *arenas, long n, uint8_t *const *out)
{
    uint8_t *C[32] = {0};
    int nc = 0;
    for (int p = k; p < k + m; ++p) {
        if (!(mask & (1u << p))) continue;
        uint8_t *res = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
        int touched = 0;
        for (int s = 0; s < k; ++s)
            if (mask & (1u << s))
                ref_recover_units(matrix, k, p, s, arenas[p], arenas[s], n, res, &touched);
        if (!touched) memcpy(res, arenas[p], (size_t)n);
        C[nc++] = res;
    }
    int r = ref_bottom_half(matrix, k, m, mask, (const uint8_t *const *)C, n, out);
    for (int i = 0; i < nc; ++i) free(C[i]);
    return r;
}
