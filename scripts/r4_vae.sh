#!/bin/bash
# LDS-DMA VAE conv: bit-identity + torch tests, then decode A/B (alternating processes, SA_CONV_DMA=0/1)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-vae}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_vae_conv_dma.py \
  > gpurun_out/t_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/t_$TAG.log | tail -8; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/kbvae_$TAG.jsonl
# a variant "D" runs SA_CONV_DMA=D; "D:0" also sets SA_RMS3=0 (the lane-padded RMS-norm kernel)
for r in 1 2; do for v in ${VARIANTS:-0 1 2}; do
  d=${v%%:*}; rms=1; [ "$v" != "$d" ] && rms=${v#*:}
  SA_CONV_DMA=$d SA_RMS3=$rms timeout -k 10 300 python scripts/kb_vae.py 3 2>/dev/null | sed "s/^{/{\"dma\": $d, \"rms3\": $rms, \"round\": $r, /" >> gpurun_out/kbvae_$TAG.jsonl
  rc=$?; [ $rc -ne 0 ] && { echo "kb_vae failed rc=$rc"; exit $rc; }
done; done
cat gpurun_out/kbvae_$TAG.jsonl
if [ -n "${PROF:-}" ]; then
  SA_CONV_DMA=$PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vaeprof_$TAG -o vp \
    -- python scripts/kb_vae.py 1 > gpurun_out/vaeprof_$TAG.log 2>&1 || { tail -5 gpurun_out/vaeprof_$TAG.log; exit 1; }
  f=$(ls gpurun_out/vaeprof_$TAG/*/vp_kernel_stats.csv gpurun_out/vaeprof_$TAG/vp_kernel_stats.csv 2>/dev/null | tail -1)
  cut -d, -f1-4 "$f" | head -12
fi
