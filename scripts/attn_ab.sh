#!/bin/bash
# attention schedule A/B on one box: the attention numerics tests, then kbench attnvar (one config-2
# self-attention launch per variant, interleaved rounds) and ditvar (30-layer DiT forwards per variant).
# usage: scripts/attn_ab.sh <tag> <variants, e.g. 1,4> [pytest -k expr]
set -u
mkdir -p gpurun_out
tag=$1; vars=$2; kexpr=${3:-attention_segments or self_attention_fullsize}
scripts/gpustep.sh 600 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 300 --timeout-method thread -k "$kexpr"
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/t_$tag.log | tail -1; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/t_$tag.log | head; exit $rc; }
SA_KB_AVARS=$vars scripts/gpustep.sh 600 gpurun_out/attn_ab_$tag.jsonl python -u -m stableavatar_amd.kbench attnvar ditvar
rc=$?; echo "kbench rc=$rc"; grep kernel gpurun_out/attn_ab_$tag.jsonl; exit $rc
