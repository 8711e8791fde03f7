#!/bin/bash
# GEMM schedule A/B: the GEMM numerics tests, then kbench gemmvar over the given kernel ids (interleaved rounds)
# usage: scripts/gemm_ab.sh <tag> <kernel ids e.g. 2,3> [shapes e.g. qkv,ffn_up] [pytest -k expr]
set -u
mkdir -p gpurun_out
tag=$1; vars=$2; shapes=${3:-}; kexpr=${4:-gemm or dit_vs_reference}
scripts/gpustep.sh 600 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 300 --timeout-method thread -k "$kexpr"
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/t_$tag.log | tail -1; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/t_$tag.log | head; exit $rc; }
SA_KB_GVARS=$vars SA_KB_SHAPES=$shapes scripts/gpustep.sh 600 gpurun_out/gemm_ab_$tag.jsonl python -u -m stableavatar_amd.kbench gemmvar
rc=$?; echo "kbench rc=$rc"; grep kernel gpurun_out/gemm_ab_$tag.jsonl; exit $rc
