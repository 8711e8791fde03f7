#!/bin/bash
# persistent GEMM start-phase stagger (SA_GEMM_STAGGER = latest phase as a fraction of one tile's K loop) vs none:
# kbench gemmvar arms "0" (auto), "0::0.25", "0::0.5", "0::1" and the no-epilogue K loop (8), interleaved rounds
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5st}
SA_KB_SHAPES=${SHAPES:-qkv,o_proj,cross_q,ffn_up,ffn_down} SA_KB_GVARS=${GVARS:-0,0::0.25,0::0.5,0::1,8} \
  timeout -k 10 400 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/gemm_stagger_$TAG.jsonl 2> gpurun_out/gemm_stagger_$TAG.err
rc=$?; cat gpurun_out/gemm_stagger_$TAG.jsonl; tail -3 gpurun_out/gemm_stagger_$TAG.err; exit $rc
