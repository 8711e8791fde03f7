#!/bin/bash
# where the bf16 GEMM epilogue's time goes: the default library vs a build whose bf16 row epilogue skips its global
# stores (SA_EPI_EXP=1: LDS-strip round trip and conversion kept) vs the K loop alone (kernel 8); two processes
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5en}
export SA_KB_SHAPES=qkv,cross_q,ffn_up SA_KB_GVARS=0,8
timeout -k 10 300 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/gemm_epi_def_$TAG.jsonl 2> gpurun_out/gemm_epi_$TAG.err
rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/gemm_epi_$TAG.err; exit $rc; }
SA_KB_NOCHECK=1 SA_LIB=build_ab/epinostore/libstableavatar_hip.so timeout -k 10 300 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/gemm_epi_nostore_$TAG.jsonl 2>> gpurun_out/gemm_epi_$TAG.err
rc=$?; cat gpurun_out/gemm_epi_def_$TAG.jsonl gpurun_out/gemm_epi_nostore_$TAG.jsonl; exit $rc
