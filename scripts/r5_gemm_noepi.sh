#!/bin/bash
# GEMM: the s9 kernel with and without its epilogue (256- and 192-row tiles) at the config-2 shapes
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5e}
SA_KB_GVARS=${GVARS:-6,8,7,9} SA_KB_SHAPES=${SHAPES:-qkv,o_proj,cross_q,ffn_up,ffn_down} timeout -k 10 400 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/kb_gemm_$TAG.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb_gemm_$TAG.jsonl; exit $rc
