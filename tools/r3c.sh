set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
tools/gpu_steps.sh r3c \
 "ops|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k 'split or sample or skinny'" \
 "wgemm|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wgemm_gpu.py" \
 "engine|900|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_continuous_gpu.py tests/test_fullsize_gpu.py" \
 "head_combine|400|python3 bench.py --steps 3 --warmup 1 --no-single" \
 "head_reduce|400|CAIN_WGEMM_COMBINE=0 python3 bench.py --steps 3 --warmup 1 --no-single" \
 "b1_qwen|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c/pq -o run -- python3 bench.py --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-energy --no-single" \
 "b1_gemma|300|python3 bench.py --model gemma:2b --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_qwen2|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_llama|300|python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single" \
 "b1_llama_fp8|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c/pf8 -o run -- python3 bench.py --batch 1 --steps 2 --warmup 1 --weights fp8 --no-single"
find gpurun_out/r3c -name "*kernel_trace.csv" -delete
