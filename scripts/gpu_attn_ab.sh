#!/bin/bash
# attention kernel A/B: numerics tests of every schedule, then interleaved timing (kbench attnvar: one
# self-attention launch at config 2; ditvar: full 30-layer DiT forwards) -> gpurun_out/attn_ab_<tag>.jsonl
set -u
mkdir -p gpurun_out
tag=${1:-x}
kexpr=${2:-attention or multi_rank}
scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 600 --timeout-method thread -k "$kexpr"
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_$tag.log; [ $rc -ne 0 ] && exit $rc
SA_KB_AVARS=${AVARS:-1} scripts/gpustep.sh 600 gpurun_out/attn_ab_$tag.jsonl python -u -m stableavatar_amd.kbench attnvar ditvar
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/attn_ab_$tag.jsonl | grep kernel; exit $rc
