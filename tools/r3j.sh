set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3j
tools/gpu_steps.sh r3j \
 "sample|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k 'sample'" \
 "front|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_front_gpu.py" \
 "trace_qwen|120|python3 tools/front_trace.py --model qwen2:1.5b --pos 700" \
 "trace_llama|120|python3 tools/front_trace.py --model llama3.1:8b --pos 700" \
 "b1_qwen_prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3j/pq -o run -- python3 bench.py --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-energy --no-single" \
 "b1_qwen|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_qwen_off|300|CAIN_FRONT=0 python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3j \
 "b1_llama|300|python3 bench.py --model llama3.1:8b --batch 1 --steps 1 --warmup 1 --no-single --no-energy" \
 "b1_llama_off|300|CAIN_FRONT=0 python3 bench.py --model llama3.1:8b --batch 1 --steps 1 --warmup 1 --no-single --no-energy"
find gpurun_out/r3j -name "*kernel_trace.csv" -delete
