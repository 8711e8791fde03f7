#!/bin/bash
# HBM traffic of the bench's own kernel launches (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in
# separate passes, FETCH_SIZE x2 on gfx950): bench.py over one clip of 2 sampling steps (60 DiT layers), counters
# on the self-attention and persistent-GEMM dispatches only.  -> gpurun_out/pmcb_<counter>/
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "attn_fwd_v6t_kernel|gemm_s8_kernel" --output-format csv \
    -d gpurun_out/pmcb_$c -o run -- python bench.py --steps 1 --warmup 0 --sample-steps 2 --no-cpu-baseline \
    --no-encode > gpurun_out/pmcb_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; tail -2 gpurun_out/pmcb_$c.log; [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_traffic.py --bench gpurun_out gpurun_out/pmc_bench_traffic.json
