#!/bin/bash
# A/B of several builds of the library on one box, alternating processes (2 rounds):
#   scripts/ab_libs.sh <tag> "<lib1> <lib2> ..." <kbench args...>
# each lib also runs scripts/res_hash.py once (output hashes for bit-identity checks).
set -u
mkdir -p gpurun_out
tag=$1; libs=$2; shift 2
for l in $libs; do
  n=$(basename "$l" .so)
  SA_LIB=$l scripts/gpustep.sh 300 gpurun_out/hash_${tag}_$n.log env PYTHONPATH=. python -u scripts/res_hash.py || exit 1
done
for i in 1 2; do
  for l in $libs; do
    n=$(basename "$l" .so)
    SA_LIB=$l scripts/gpustep.sh 400 gpurun_out/ab_${tag}_${n}_$i.log python -u -m stableavatar_amd.kbench "$@" || exit 1
  done
done
for f in gpurun_out/hash_${tag}_*.log; do echo "== $f"; grep hash "$f"; done
for f in gpurun_out/ab_${tag}_*.log; do echo "== $f"; grep kernel "$f"; done
