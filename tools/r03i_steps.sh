# round-3 rocprofv3 evidence on the final kernels: kernel-trace + FETCH_SIZE / WRITE_SIZE
# passes per workload, default (PERM) engine, then the LDS engine for the metric and the
# diff-update
set -e
bash tools/profile_round.sh r03
PROF_ENGINE=lds PROF_WORKLOADS="rs32_4k rs32_diff_update" bash tools/profile_round.sh r03_lds
