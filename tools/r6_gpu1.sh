#!/usr/bin/env bash
# round 6: native GGUF Q4 kernel tests and batch-1 rates, then the wide GEMM's in-launch split-K combine
# (tests + headline A/B)
set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_q4_gpu.py > gpurun_out/r6w/q4_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6w/q4_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # a failed assertion (1) still lets the next steps run; a crash does not
timeout -k 10 300 python tools/b1_ab.py --models llama3.1:8b,qwen2:1.5b,gemma:2b --dtype fp4,q4_k,q4_0 --label q4 --out gpurun_out/r6w/b1_q4.jsonl || exit 1
bash tools/wg_inline_ab.sh
