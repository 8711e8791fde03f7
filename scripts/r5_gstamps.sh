#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5gs}
SA_LIB=build_ab/gstamps/libstableavatar_hip.so timeout -k 10 300 python -u scripts/gemm_stamps.py > gpurun_out/gemm_stamps_$TAG.jsonl 2> gpurun_out/gemm_stamps_$TAG.err
rc=$?; cat gpurun_out/gemm_stamps_$TAG.jsonl; tail -3 gpurun_out/gemm_stamps_$TAG.err; exit $rc
