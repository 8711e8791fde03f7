#!/bin/bash
# Stall anatomy of the attention and GEMM kernels: one SQ pass (8 counters) + GRBM_GUI_ACTIVE.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- python -m stableavatar_amd.kbench attn1 gemm1 > gpurun_out/pmc_sq.log 2>&1
echo "pmc sq rc=$?"
