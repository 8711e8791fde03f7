#!/bin/bash
# A/B of two builds of the library on one box: build_ab/lib_head.so (baseline) vs the in-tree library,
# alternating processes.  usage: scripts/ab_lib.sh <tag> <pytest -k expr or -> <kbench args...>
set -u
mkdir -p gpurun_out
tag=$1; kexpr=$2; shift 2
if [ "$kexpr" != "-" ]; then
  scripts/gpustep.sh 600 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 300 --timeout-method thread -k "$kexpr" || { tail -30 gpurun_out/t_$tag.log; exit 1; }
  tail -2 gpurun_out/t_$tag.log
fi
for i in 1 2; do
  SA_LIB=build_ab/lib_head.so scripts/gpustep.sh 400 gpurun_out/ab_${tag}_head_$i.log python -u -m stableavatar_amd.kbench "$@" || exit 1
  scripts/gpustep.sh 400 gpurun_out/ab_${tag}_new_$i.log python -u -m stableavatar_amd.kbench "$@" || exit 1
done
for f in gpurun_out/ab_${tag}_*.log; do echo "== $f"; grep kernel "$f"; done
