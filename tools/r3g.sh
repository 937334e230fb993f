set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3g
tools/gpu_steps.sh r3g \
 "ops|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k 'sample'" \
 "b1_qwen|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3g/pq -o run -- python3 bench.py --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-energy --no-single" \
 "b1_qwen2|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single" \
 "engine|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_continuous_gpu.py"
find gpurun_out/r3g -name "*kernel_trace.csv" -delete
