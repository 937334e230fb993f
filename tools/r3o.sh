set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3o \
 "trace|500|python3 tools/wgemm_trace.py --model llama3.1:8b --variants 0,5" \
 "attn|300|python3 tools/bench_kernels.py --attn-only --attn 256:350,256:700,256:1400,1:700"
