#!/bin/bash
# round 4 GPU check: selected -m gpu tests (args: pytest node ids / -k expr), then optional extra step
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error|rel|bit-identical|PASS|FAIL" gpurun_out/gpu_tests_$TAG.log | tail -60
echo "pytest rc=$rc"
exit $rc
