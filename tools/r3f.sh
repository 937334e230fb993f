set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3f
tools/gpu_steps.sh r3f \
 "ops|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k 'sample or split'" \
 "b1_qwen|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/pq -o run -- python3 bench.py --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-energy --no-single" \
 "b1_qwen2|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_gemma|300|python3 bench.py --model gemma:2b --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_llama|300|python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single" \
 "head|400|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/ph -o run -- python3 bench.py --steps 1 --warmup 1 --no-single --no-energy"
find gpurun_out/r3f -name "*kernel_trace.csv" -delete
