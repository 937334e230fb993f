set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ad \
 "test|300|python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k 'skinny_split'" \
 "full2|500|CAIN_SKINNY_SPLIT=2 python -u -m pytest tests/test_fullsize_gpu.py -k logits_match_oracle -x -q --timeout 400 --timeout-method thread" \
 "l1|300|$B" \
 "l2|300|CAIN_SKINNY_SPLIT=2 $B" \
 "l1b|300|$B" \
 "l2b|300|CAIN_SKINNY_SPLIT=2 $B" \
 "q1|300|$B --model qwen2:7b" \
 "q2|300|CAIN_SKINNY_SPLIT=2 $B --model qwen2:7b" \
 "prof|300|CAIN_SKINNY_SPLIT=2 bash tools/prof_bench.sh r3ad/prof_b1_llama_split2 --batch 1 --steps 1 --warmup 1 --no-single --no-energy"
