#!/bin/bash
# VAE conv schedule A/B: VAE numerics tests on a candidate library, then the config-2 decode
# (scripts/kb_vae.py: ms + output checksum) alternating processes over the libraries.
#   scripts/gpu_conv_ab.sh <tag> <test lib> "<lib1> <lib2> ..."
set -u
mkdir -p gpurun_out
tag=$1; tlib=$2; libs=$3
SA_LIB=$tlib scripts/gpustep.sh 600 gpurun_out/t_$tag.log python -u -m pytest tests/test_gpu_vae_pipeline.py -m gpu -v -x --timeout 300 --timeout-method thread || { tail -30 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
for i in 1 2; do
  for l in $libs; do
    n=$(basename "$l" .so)
    SA_LIB=$l scripts/gpustep.sh 300 gpurun_out/kbvae_${tag}_${n}_$i.log python -u scripts/kb_vae.py 3 || exit 1
  done
done
for f in gpurun_out/kbvae_${tag}_*.log; do echo "== $f"; grep kernel "$f"; done
