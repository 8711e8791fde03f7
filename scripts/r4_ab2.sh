#!/bin/bash
# A/B of build_ab/old/libstableavatar_hip.so vs the in-tree library: output hashes, then kbench (alternating)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
SA_LIB=build_ab/old/libstableavatar_hip.so timeout -k 10 120 python scripts/gemm_hash.py > gpurun_out/hash_${TAG}_old.log 2>&1 || exit 1
timeout -k 10 120 python scripts/gemm_hash.py > gpurun_out/hash_${TAG}_new.log 2>&1 || exit 1
diff <(grep -v amdgpu gpurun_out/hash_${TAG}_old.log) <(grep -v amdgpu gpurun_out/hash_${TAG}_new.log) && echo "HASHES IDENTICAL"
for i in 1 2; do
  SA_LIB=build_ab/old/libstableavatar_hip.so timeout -k 10 300 python -m stableavatar_amd.kbench "$@" > gpurun_out/ab_${TAG}_old_$i.log 2>&1 || exit 1
  timeout -k 10 300 python -m stableavatar_amd.kbench "$@" > gpurun_out/ab_${TAG}_new_$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_${TAG}_*.log; do echo "== $f"; grep kernel "$f" | cut -c1-250; done
