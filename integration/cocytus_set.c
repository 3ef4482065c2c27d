/*
 * integration/cocytus_set.c -- the data process's SET diffs batched (see cocytus_set.h).
 */
#include "cocytus_set.h"

#include <stdlib.h>

int cocytus_set_diffs_gf(struct ecmem *ecm, const cocytus_set_diff *sets, int n, void *stream) {
    if (!ecm || n < 0 || (n && !sets)) return CEC_EINVAL;
    if (n == 0) return CEC_OK;
    cec_region_job *jobs = malloc(sizeof *jobs * (size_t)n);
    if (!jobs) return CEC_ENOMEM;
    for (int i = 0; i < n; ++i) {
        if (sets[i].nbytes && (!sets[i].value || !sets[i].diff)) {
            free(jobs);
            return CEC_EINVAL;
        }
        /* memcached.c:2678-2681: diff = new, then diff ^= 1 * old: one job, the old bytes
         * as its base (diff = old ^ 1 * new; XOR commutes) */
        jobs[i].src = sets[i].value;
        jobs[i].dst = sets[i].diff;
        jobs[i].base = ecmem_get(ecm, sets[i].addr);
        jobs[i].len = sets[i].nbytes;
        jobs[i].multby = 1;
        jobs[i].add = 1;
    }
    const int rc = cec_region_multiply_batch(jobs, n, stream);
    free(jobs);
    return rc;
}
