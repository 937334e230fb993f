set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
A="python3 tools/bench_kernels.py --attn-only --attn 256:350,256:700,256:1400"
tools/gpu_steps.sh r3y \
 "test|400|python -u -m pytest tests/test_ops_gpu.py tests/test_w8a8_gpu.py tests/test_kv8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "attn0|200|CAIN_ATTN_RING=0 $A" \
 "attn1|200|$A" \
 "b_ring|300|$B" \
 "b_reg|300|CAIN_ATTN_RING=0 $B" \
 "b_ringb|300|$B" \
 "b_split|300|CAIN_SAMPLE_SPLIT_MAX=256 $B" \
 "b_fp8|300|$B --weights fp8 --kv fp8"
