#!/bin/bash
# full GPU suite + __graft_entry__.smoke() on the current tree (stops at a fault)
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 1000 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 5 --timeout 600 --timeout-method thread
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/t_$tag.log | tail -1; [ $rc -eq 99 ] && exit 99
scripts/gpustep.sh 300 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()"
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke_$tag.log
exit $(( rc | rc2 ))
