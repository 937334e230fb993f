set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
A="python3 tools/bench_kernels.py --attn-only --attn 256:350,256:700,256:1400"
tools/gpu_steps.sh r3w \
 "test|240|python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention_ring or attention_many_rows'" \
 "attn0|200|$A" \
 "attn1|200|CAIN_ATTN_RING=1 $A" \
 "attn2|200|CAIN_ATTN_RING=2 $A" \
 "attn3|200|CAIN_ATTN_RING=3 $A" \
 "b0|300|$B" \
 "b1|300|CAIN_ATTN_RING=1 $B" \
 "b2|300|CAIN_ATTN_RING=2 $B" \
 "b3|300|CAIN_ATTN_RING=3 $B" \
 "b0b|300|$B"
