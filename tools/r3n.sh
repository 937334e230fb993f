set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
tools/gpu_steps.sh r3n \
 "sample|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k 'sample'" \
 "strace|300|python3 tools/sample_trace.py --model qwen2:1.5b" \
 "engine|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_continuous_gpu.py" \
 "b1_qwen|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_qwen_off|300|CAIN_FRONT=0 python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
