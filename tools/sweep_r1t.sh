#!/bin/bash
# Batched GEMM epilogue: grouped epilogue-input loads (one round trip per 8 row blocks instead of per block).
set -o pipefail
mkdir -p gpurun_out/r1t
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r1t/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r1t/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python tools/bench_kernels.py --rows 64,128,256 --roles qkv,o,gateup,down,lm_head --gemm-only --norm --waves 0 > gpurun_out/r1t/k.jsonl 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/r1t/k.jsonl'):
    if l.startswith('{'):
        r=json.loads(l)
        if r['path']=='batched': print('  ',r['role'],r['M'],r['us'],r['TBps'])
"
timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/r1t/bench.log 2>&1 || exit 1
echo "bench $(tail -1 gpurun_out/r1t/bench.log | cut -c60-130)"
mkdir -p gpurun_out/r1t/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1t/prof -o run -- python3 bench.py --no-energy --words 300 --steps 1 --warmup 0 > gpurun_out/r1t/prof/bench.log 2>&1 || exit 1
find gpurun_out/r1t/prof -name "*kernel_trace.csv" -delete
cut -c1-80,130-175 gpurun_out/r1t/prof/run_kernel_stats.csv | head -8
