set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3s \
 "trace|400|python3 tools/wgemm_trace.py --model llama3.1:8b --variants 0,19 --only qkv,o,down" \
 "b_v0|300|$B" \
 "b_v19|300|CAIN_WGEMM_VARIANT=19 $B" \
 "b_v0b|300|$B" \
 "b_v19b|300|CAIN_WGEMM_VARIANT=19 $B"
