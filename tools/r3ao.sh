set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ao \
 "test|400|python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 250 --timeout-method thread" \
 "l|300|$B" \
 "l0|300|CAIN_SKINNY_W4=0 $B"
