#!/bin/bash
# v13 build variants A/B (kbench attnvar, kernel 5) against the default library's v6t / v13
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5u}
for rnd in 1 2; do
  SA_KB_AVARS=3,5 timeout -k 10 200 python -u -m stableavatar_amd.kbench attnvar 2>/dev/null | sed "s/^{/{\"lib\": \"default\", /" >> gpurun_out/kb_v13var_$TAG.jsonl || exit 1
  for v in ${VARS:-noprio dmafirst both}; do
    SA_LIB=build_ab/$v/libstableavatar_hip.so SA_KB_AVARS=5 timeout -k 10 200 python -u -m stableavatar_amd.kbench attnvar 2>/dev/null | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/kb_v13var_$TAG.jsonl || exit 1
  done
done
cut -c1-60,150-400 gpurun_out/kb_v13var_$TAG.jsonl
