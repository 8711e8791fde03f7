#!/bin/bash
# round 5: V^T self-attention path -- kernel + DiT parity tests, then the bench with and without the kernel timer
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -v -s --timeout 300 --timeout-method thread -k "transposed or attention or vt_attention or block_fullsize" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|rel-L2|bit-identical" gpurun_out/tests_$TAG.log | tail -12; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 400 python3 bench.py --gpus 1 --steps ${STEPS:-2} --warmup 1 --no-cpu-config1 --no-encode > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], json.dumps(d.get('kernels'))[:1500])"
if [ -n "${KTOFF:-}" ]; then
  SA_BENCH_KTIMER=0 timeout -k 10 400 python3 bench.py --gpus 1 --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-encode > gpurun_out/bench_${TAG}_kt0.json 2> gpurun_out/bench_${TAG}_kt0.err
  rc=$?; echo "bench kt0 rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_kt0.json')); print('kt0', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
fi
exit $rc
