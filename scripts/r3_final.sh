#!/bin/bash
# Round-3 final measurement: the driver's bench command (--steps 20 --warmup 5, CPU baseline child included)
# with its wall time, a rocprofv3 kernel-trace/stats run of one clip, and one SQ PMC pass over the bench's own
# self-attention and VAE conv launches (2 sampling steps + the decode).  Stops at the first failure.
set -u
mkdir -p gpurun_out
tag=${1:-r3f}
t0=$(date +%s)
scripts/gpustep.sh 600 gpurun_out/bench_$tag.log python -u bench.py --steps 20 --warmup 5
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - t0 ))s"; tail -c 300 gpurun_out/bench_$tag.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-encode > gpurun_out/prof_$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "attn_fwd_v6_kernel|conv3d_cl_kernel|attn_cross3_kernel" --kernel-trace --output-format csv -d gpurun_out/pmc_sq_$tag -o run -- python bench.py --steps 1 --warmup 0 --sample-steps 2 --no-cpu-baseline --no-encode > gpurun_out/pmc_sq_$tag.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/pmc_sq_$tag -name run_counter_collection.csv -print -quit)
[ -n "$f" ] && python3 scripts/pmc_table.py "$(dirname "$f")" 50 > gpurun_out/pmc_sq_$tag.txt 2>&1
tail -5 gpurun_out/pmc_sq_$tag.txt
exit 0
