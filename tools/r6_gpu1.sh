#!/usr/bin/env bash
# round 6: native GGUF Q4 kernel tests, then the wide GEMM's in-launch split-K combine (tests + headline A/B)
set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_q4_gpu.py > gpurun_out/r6w/q4_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r6w/q4_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # a failed assertion (1) still lets the wgemm step run; a crash does not
bash tools/wg_inline_ab.sh
