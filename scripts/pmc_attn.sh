#!/bin/bash
# HBM traffic of the self-attention kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in
# separate passes; FETCH_SIZE x2 on gfx950) + the counter list of this box.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$c -o run -- python -m stableavatar_amd.kbench attn1 > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done

python3 scripts/pmc_traffic.py gpurun_out gpurun_out/pmc_attn_traffic.json
