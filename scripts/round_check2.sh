#!/bin/bash
# Round-end style GPU check: all GPU tests, smoke() both as the driver calls it and after an in-process
# build, attention HBM-traffic PMC passes, bench, rocprof kernel stats.  Stops at the first fault.
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 700 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 200 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()"
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 300 gpurun_out/smoke2_$tag.log python __graft_entry__.py smoke
rc=$?; echo "smoke(build) rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/pmc_attn.sh > gpurun_out/pmcattn_$tag.log 2>&1; rc=$?; echo "pmc attn rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 300 gpurun_out/bench_$tag.log python bench.py; rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py > gpurun_out/prof_$tag.log 2>&1
echo "prof rc=$?"
