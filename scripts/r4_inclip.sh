#!/bin/bash
# in-clip kernel stats (2 sampling steps = 60 DiT layers) for SA_GEMM_SCHED 8 and 9, then one SQ + clock PMC pass
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4c}
for sc in ${SCHEDS:-8 9}; do
  SA_GEMM_SCHED=$sc timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ic_${TAG}_s$sc -o run -- \
    python bench.py --steps 1 --warmup 1 --sample-steps 4 --no-cpu-baseline --no-encode > gpurun_out/ic_${TAG}_s$sc.log 2>&1
  rc=$?; echo "sched $sc rc=$rc"; tail -1 gpurun_out/ic_${TAG}_s$sc.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
if [ -n "${PMC:-}" ]; then
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex "attn_fwd_v6_kernel|gemm_s8_kernel|attn_cross3" \
    --kernel-trace --output-format csv -d gpurun_out/icpmc_$TAG -o run -- python bench.py --steps 1 --warmup 0 \
    --sample-steps 2 --no-cpu-baseline --no-encode > gpurun_out/icpmc_$TAG.log 2>&1
  rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_table.py gpurun_out/icpmc_$TAG 100 > gpurun_out/icpmc_$TAG.txt
fi
exit 0
