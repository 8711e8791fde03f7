#!/bin/bash
# SQ stall anatomy of the V^T self-attention (kbench attnvar, AVARS; profiles/r05 pmc_sq_attn_v6t_r5y.json, profiles/r06
# pmc_sq_attn_v6t_r6.json): one SQ pass of 8 counters + GRBM
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r6}
SA_KB_AVARS=${AVARS:-3} timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "attn_fwd" --output-format csv -d gpurun_out/pmc_attn_$TAG -o run -- python -m stableavatar_amd.kbench attnvar > gpurun_out/pmc_attn_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/pmc_attn_$TAG -name "*counter_collection.csv" | head -1); echo "$f"
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
