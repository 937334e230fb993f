set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3q \
 "trace|400|python3 tools/wgemm_trace.py --model llama3.1:8b --variants 0,10,12,14,15,16 --only gateup,lm_head" \
 "b_v0|300|python3 bench.py --steps 2 --warmup 1 --no-single --no-energy" \
 "b_v14|300|CAIN_WGEMM_VARIANT=14 python3 bench.py --steps 2 --warmup 1 --no-single --no-energy" \
 "b_v12|300|CAIN_WGEMM_VARIANT=12 python3 bench.py --steps 2 --warmup 1 --no-single --no-energy" \
 "b_v10|300|CAIN_WGEMM_VARIANT=10 python3 bench.py --steps 2 --warmup 1 --no-single --no-energy" \
 "b_v0b|300|python3 bench.py --steps 2 --warmup 1 --no-single --no-energy"
