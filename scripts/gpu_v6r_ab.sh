#!/bin/bash
# register-staged self-attention (kernel 3) vs the LDS-DMA one (kernel 1): numerics, then interleaved timing
set -u
mkdir -p gpurun_out
tag=${1:-v6r}
scripts/gpustep.sh 600 gpurun_out/t_$tag.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -v -x --timeout 300 --timeout-method thread -k "attention_segments or self_attention_fullsize" || { tail -30 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
SA_KB_AVARS=1,3 scripts/gpustep.sh 600 gpurun_out/attn_ab_$tag.jsonl python -u -m stableavatar_amd.kbench attnvar ditvar attnvar || exit 1
grep kernel gpurun_out/attn_ab_$tag.jsonl
