set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3h
tools/gpu_steps.sh r3h \
 "front|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_front_gpu.py" \
 "engine|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_continuous_gpu.py" \
 "b1_qwen_prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h/pq -o run -- python3 bench.py --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-energy --no-single" \
 "b1_qwen|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_qwen_off|300|CAIN_FRONT=0 python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_llama|300|python3 bench.py --model llama3.1:8b --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
find gpurun_out/r3h -name "*kernel_trace.csv" -delete
