#!/bin/bash
# rocprofv3 kernel stats of one Ulysses rank's forward (scripts/sp_rank_compute.py) at degrees 1, 4 and 8
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for n in ${SP_DEGREES:-1 4 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sp$n -o run -- python3 -u $R/scripts/sp_rank_compute.py $n > $R/gpurun_out/prof_sp$n.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/prof_sp$n -name "run_kernel_stats.csv" | head -1)
  python3 $R/scripts/prof_summary.py "$f" $R/gpurun_out/sp_rank_kernels_n$n.csv
done
