set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3r \
 "trace|400|python3 tools/wgemm_trace.py --model llama3.1:8b --variants 0,17 --only qkv,o,gateup,down" \
 "b_v0|300|$B" \
 "b_v17|300|CAIN_WGEMM_VARIANT=17 $B" \
 "b_v18|300|CAIN_WGEMM_VARIANT=18 $B" \
 "b_v14|300|CAIN_WGEMM_VARIANT=14 $B" \
 "b_v0b|300|$B" \
 "b_v17b|300|CAIN_WGEMM_VARIANT=17 $B"
