set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
tools/gpu_steps.sh r3d \
 "ops|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py" \
 "b1_qwen|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/pq -o run -- python3 bench.py --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-energy --no-single" \
 "b1_qwen2|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_gemma|300|python3 bench.py --model gemma:2b --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_llama|300|python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_llama_fp8|300|python3 bench.py --batch 1 --steps 2 --warmup 1 --weights fp8 --no-single" \
 "numerics|1100|python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_w8a8_gpu.py tests/test_continuous_gpu.py"
find gpurun_out/r3d -name "*kernel_trace.csv" -delete
