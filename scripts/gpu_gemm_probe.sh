#!/bin/bash
# rocprofv3 passes over scripts/gemm_probe.py (hipBLASLt vs our persistent GEMM): kernel trace + stats,
# one SQ pass (stall anatomy + MFMA busy + clock), one L2 pass, one FETCH_SIZE pass -- each its own run
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/gprobe; mkdir -p $o
shapes=${1:-cross_q,ffn_up}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o run -- python3 scripts/gemm_probe.py $shapes > $o/kt.log 2>&1 || exit 99
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $o/sq -o run -- python3 scripts/gemm_probe.py $shapes > $o/sq.log 2>&1 || exit 99
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $o/l2 -o run -- python3 scripts/gemm_probe.py $shapes > $o/l2.log 2>&1 || exit 99
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $o/fs -o run -- python3 scripts/gemm_probe.py $shapes > $o/fs.log 2>&1 || exit 99
for p in sq l2 fs; do echo "== $p"; python3 scripts/pmc_table.py $(dirname $(find $o/$p -name run_counter_collection.csv | head -1)) 100; done
