set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
F="python3 bench.py --batch 1 --weights fp8 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ai \
 "test|300|CAIN_SKINNY_XLDS=1 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k 'skinny or graph_replay or oracle or chunk_max'" \
 "full|300|CAIN_SKINNY_XLDS=1 python -u -m pytest tests/test_fullsize_gpu.py -k logits_match_oracle -x -q --timeout 250 --timeout-method thread" \
 "l0|300|$B" \
 "l1|300|CAIN_SKINNY_XLDS=1 $B" \
 "l0b|300|$B" \
 "l1b|300|CAIN_SKINNY_XLDS=1 $B" \
 "q0|300|$B --model qwen2:1.5b" \
 "q1|300|CAIN_SKINNY_XLDS=1 $B --model qwen2:1.5b" \
 "g0|300|$B --model gemma:2b" \
 "g1|300|CAIN_SKINNY_XLDS=1 $B --model gemma:2b" \
 "f_u2|300|$F" \
 "f_u4|300|CAIN_W8_U=4 $F" \
 "prof|300|CAIN_SKINNY_XLDS=1 bash tools/prof_bench.sh r3ai/prof_b1_llama_xl --batch 1 --steps 1 --warmup 1 --no-single --no-energy"
