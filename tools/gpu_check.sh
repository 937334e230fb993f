#!/bin/bash
# GPU verification pass: kernels + engine tests, smoke, short bench. Each GPU step bounded; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m "${PYTEST_MARK:-gpu}" -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -20 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -20 gpurun_out/bench.log; exit $rc
