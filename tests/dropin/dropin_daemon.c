/*
 * tests/dropin/dropin_daemon.c -- the drop-in under memcached's start-up order.
 *
 * memcached builds the coding matrix in main() (memcached.c:6845) BEFORE it
 * daemonizes (memcached.c:6946-6955: fork(), the parent exits, the child serves).
 * The GPU is only usable in the process that opened it, so the shim's host-only
 * symbols (reed_sol_*, jerasure_invert_matrix, galois_single_*) must not touch the
 * GPU, and the first galois_w08_region_multiply -- in the daemon child -- must.
 * This program does exactly that order: matrix + inversion in the parent, fork(),
 * then region multiplies in the child (pageable 4 KiB values like c->vbuf, and an
 * odd-length one like vlen + 2), checked byte by byte against galois_single_multiply.
 * The parent waits for the child instead of exiting, to report its status.
 */
#include <galois.h>
#include <jerasure.h>
#include <reed_sol.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

static int child_work(const int *matrix, int K) {
    int bad = 0;
    const int sizes[2] = {4096, 4098};
    for (int t = 0; t < 2; ++t) {
        const int n = sizes[t];
        char *region = malloc(n), *r2 = malloc(n), *exp = malloc(n);
        unsigned s = 12345u + (unsigned)t;
        for (int i = 0; i < n; ++i) {
            s = s * 1103515245u + 12345u;
            region[i] = (char)(s >> 16);
            s = s * 1103515245u + 12345u;
            r2[i] = (char)(s >> 16);
        }
        const int c = matrix[(K + 1) * K + 1]; /* a non-trivial coefficient (245 for RS(3,2)) */
        for (int i = 0; i < n; ++i)
            exp[i] = (char)(r2[i] ^ galois_single_multiply((unsigned char)region[i], c, 8));
        galois_w08_region_multiply(region, c, n, r2, 1);
        for (int i = 0; i < n; ++i) bad += r2[i] != exp[i];
        free(region);
        free(r2);
        free(exp);
    }
    printf("child %d mismatches\n", bad);
    fflush(stdout);
    return bad ? 1 : 0;
}

int main(void) {
    const int K = 3, M = 2;
    int *matrix = reed_sol_big_vandermonde_distribution_matrix(K + M, K, 8); /* :6845 */
    if (!matrix) return 3;
    int sub[4] = {matrix[K * K + 0], matrix[K * K + 1], matrix[(K + 1) * K + 0],
                  matrix[(K + 1) * K + 1]};
    int inv[4];
    if (jerasure_invert_matrix(sub, inv, 2, 8) != 0) return 4; /* :7907, host only */
    fflush(stdout);
    const pid_t pid = fork(); /* daemonize(), memcached.c:6948-6955 */
    if (pid < 0) return 5;
    if (pid == 0) _exit(child_work(matrix, K));
    int st = 0;
    if (waitpid(pid, &st, 0) != pid) return 6;
    free(matrix);
    if (!WIFEXITED(st)) {
        fprintf(stderr, "daemon child died (status %d)\n", st);
        return 7;
    }
    return WEXITSTATUS(st);
}
