set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3as \
 "test|300|CAIN_SKINNY_W4X=8 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k 'skinny or oracle or graph_replay'" \
 "p|300|$B --model phi3:3.8b" \
 "p8|300|CAIN_SKINNY_W4X=8 $B --model phi3:3.8b" \
 "g|300|$B --model gemma:7b" \
 "g8|300|CAIN_SKINNY_W4X=8 $B --model gemma:7b" \
 "g2|300|$B --model gemma:2b" \
 "g28|300|CAIN_SKINNY_W4X=8 $B --model gemma:2b" \
 "l|300|$B" \
 "l8|300|CAIN_SKINNY_W4X=8 $B"
