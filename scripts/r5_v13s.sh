#!/bin/bash
# v13 kernel tests + A/B vs v6t, then the phase anatomy from the SA_V13_STAMPS build
set -u
TAG=${TAG:-r5r}
bash scripts/r5_v13.sh || exit $?
cd "$GRAFT_REPO_ROOT"
SA_LIB=build_ab/stamps/libstableavatar_hip.so timeout -k 10 120 python -u scripts/v13_stamps.py > gpurun_out/v13_stamps_$TAG.json 2>gpurun_out/v13_stamps_$TAG.err
rc=$?; cat gpurun_out/v13_stamps_$TAG.json; tail -3 gpurun_out/v13_stamps_$TAG.err; exit $rc
