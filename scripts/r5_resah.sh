#!/bin/bash
# fp32 gated-residual epilogue prefetch depth (SA_RES_AH: residual loads in flight per lane, default 8) A/B:
# kbench gemmvar o_proj / ffn_down in alternating processes over the default, ah12 and ah16 builds
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5ah}
export SA_KB_SHAPES=o_proj,ffn_down SA_KB_GVARS=0
for r in 1 2; do
  for L in def ah12 ah16; do
    if [ $L = def ]; then unset SA_LIB; else export SA_LIB=build_ab/$L/libstableavatar_hip.so; fi
    timeout -k 10 200 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/gemm_resah_$TAG.err | sed "s/^{/{\"lib\": \"$L\", /" >> gpurun_out/gemm_resah_$TAG.jsonl || exit 1
  done
done
cat gpurun_out/gemm_resah_$TAG.jsonl
