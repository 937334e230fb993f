set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3p \
 "trace|500|python3 tools/wgemm_trace.py --model llama3.1:8b --variants 0,10,11,12,13 --only qkv,o,gateup,down"
