#!/bin/bash
# Double-buffered LDS fragments in the batched GEMM: correctness, 32/64/128-row sweep, bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q -k "gemm or qkv" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1c.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1c.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/sweep_r1c.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-32,64,128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_D=0 || exit 1
ROWS=128 run CAIN_BGEMM_D=4 || exit 1
ROWS=128 run CAIN_BGEMM_D=6 || exit 1
ROWS=128 run CAIN_BGEMM_W=8 || exit 1
ROWS=128 run CAIN_BGEMM_W=4 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r1c.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1c.log; exit $rc
