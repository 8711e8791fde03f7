#!/bin/bash
# HBM traffic of the DiT GEMMs (one launch per shape, kbench gemm1): FETCH_SIZE and WRITE_SIZE in
# separate passes (MI355X_MICROARCH.md HBM section; FETCH_SIZE x2 on gfx950).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmcg_$c -o run -- python -m stableavatar_amd.kbench gemm1 > gpurun_out/pmcg_$c.log 2>&1
  rc=$?; echo "pmc gemm $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
