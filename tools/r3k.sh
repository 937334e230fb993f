set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3k
tools/gpu_steps.sh r3k \
 "sample|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k 'sample'" \
 "strace|300|python3 tools/sample_trace.py --model qwen2:1.5b"
