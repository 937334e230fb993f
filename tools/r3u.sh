set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3u \
 "def|300|$B" \
 "o8|300|CAIN_WGEMM_PLANS=4096:4096:256:8 $B" \
 "q5o8|300|CAIN_WGEMM_PLANS=6144:4096:256:5,4096:4096:256:8 $B" \
 "defb|300|$B" \
 "o8b|300|CAIN_WGEMM_PLANS=4096:4096:256:8 $B" \
 "q5o8b|300|CAIN_WGEMM_PLANS=6144:4096:256:5,4096:4096:256:8 $B"
