#!/bin/bash
# 16-B sc1 split-K slabs: correctness, then k-split / workgroup-target sweep at 64 and 128 rows, bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1f.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/sweep_r1f.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-64,128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_WG=0 || exit 1
run CAIN_BGEMM_WG=256 || exit 1
run CAIN_BGEMM_WG=256 CAIN_BGEMM_KSMAX=16 || exit 1
run CAIN_BGEMM_WG=512 CAIN_BGEMM_KSMAX=16 || exit 1
ROWS=128 run CAIN_BGEMM_D=4 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r1f.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1f.log; exit $rc
