#!/bin/bash
# GEMM schedule A/B in one process (kbench gemmvar): SA_KB_GVARS variants, all DiT shapes
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4g}
timeout -k 10 ${KB_TIMEOUT:-300} python -m stableavatar_amd.kbench gemmvar > gpurun_out/kb_$TAG.jsonl 2> gpurun_out/kb_$TAG.err
rc=$?; cat gpurun_out/kb_$TAG.jsonl; tail -3 gpurun_out/kb_$TAG.err; exit $rc
