#!/bin/bash
# s10 decomposition: default lib (s9 192-row with / without epilogue, s10), exp1 (no deferred stores), exp2 (no stash)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5k}
SH=${SHAPES:-cross_q,o_proj,qkv}
SA_KB_GVARS=7,9,10 SA_KB_SHAPES=$SH timeout -k 10 300 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/kb_gemm_${TAG}_def.jsonl 2>&1 || exit $?
for e in exp1 exp2; do
SA_LIB=build_ab/$e/libstableavatar_hip.so SA_KB_GVARS=10 SA_KB_SHAPES=$SH timeout -k 10 300 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/kb_gemm_${TAG}_$e.jsonl 2>&1 || exit $?
done
grep -hv amdgpu.ids gpurun_out/kb_gemm_${TAG}_*.jsonl
