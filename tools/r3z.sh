set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
A="python3 tools/bench_kernels.py --attn-only --attn 256:100,256:350,256:700,256:1400"
tools/gpu_steps.sh r3z \
 "test|300|python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention'" \
 "attn0|200|CAIN_ATTN_RING=0 $A" \
 "attn1|200|$A" \
 "b_ring|300|$B" \
 "b_reg|300|CAIN_ATTN_RING=0 $B" \
 "b_ringb|300|$B"
