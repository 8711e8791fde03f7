#!/bin/bash
# cross-attention overhead anatomy (kbench cross3, config-2 launch): default vs measurement builds that run the
# block stream twice per tile (x3r2), skip the Q load (x3noq), or both; interleaved, two rounds
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5x}
for rnd in 1 2; do
  for lib in default x3r2 x3noq x3r2noq; do
    if [ $lib = default ]; then unset SA_LIB; else export SA_LIB=build_ab/$lib/libstableavatar_hip.so; fi
    echo -n "{\"lib\": \"$lib\", \"round\": $rnd, \"r\": " >> gpurun_out/x3exp_$TAG.jsonl
    timeout -k 10 120 python -u -m stableavatar_amd.kbench cross3 2>>gpurun_out/x3exp_$TAG.err | tail -1 | tr -d '\n' >> gpurun_out/x3exp_$TAG.jsonl
    rc=$?; echo "}" >> gpurun_out/x3exp_$TAG.jsonl; [ $rc -ne 0 ] && exit $rc
  done
done
cat gpurun_out/x3exp_$TAG.jsonl
