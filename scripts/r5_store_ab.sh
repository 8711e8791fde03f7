#!/bin/bash
# GEMM output store cache policy A/B (kbench gemmvar, auto kernel): default (bf16 nt, fp32 plain) vs sc1 / sc1+nt /
# nt-everywhere builds of gemm.hip (SA_STORE_POLICY); interleaved processes, two rounds; then FETCH_SIZE of one launch
# per shape (kbench gemm1) for default and sc1
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5s}
export SA_KB_GVARS=0 SA_KB_SHAPES=qkv,o_proj,cross_q,ffn_up,ffn_down
for rnd in 1 2; do
  for lib in default stsc1 stsc1nt stnt; do
    if [ $lib = default ]; then unset SA_LIB; else export SA_LIB=build_ab/$lib/libstableavatar_hip.so; fi
    timeout -k 10 180 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/store_ab_$TAG.err | sed "s/^{/{\"lib\": \"$lib\", \"round\": $rnd, /" >> gpurun_out/store_ab_$TAG.jsonl
    rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
for lib in default stsc1; do
  if [ $lib = default ]; then unset SA_LIB; else export SA_LIB=build_ab/$lib/libstableavatar_hip.so; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_store_$lib -o run -- python -m stableavatar_amd.kbench gemm1 > gpurun_out/pmc_store_$lib.log 2>&1
  rc=$?; echo "pmc $lib rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
