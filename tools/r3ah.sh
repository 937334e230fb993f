set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --weights fp8 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ah \
 "test|300|CAIN_W8_XLDS=1 python -u -m pytest tests/test_w8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "l0|300|$B" \
 "l1|300|CAIN_W8_XLDS=1 $B" \
 "l0b|300|$B" \
 "l1b|300|CAIN_W8_XLDS=1 $B" \
 "q0|300|$B --model qwen2:1.5b" \
 "q1|300|CAIN_W8_XLDS=1 $B --model qwen2:1.5b" \
 "prof|300|CAIN_W8_XLDS=1 bash tools/prof_bench.sh r3ah/prof_b1_llama_fp8_xl --batch 1 --weights fp8 --steps 1 --warmup 1 --no-single --no-energy"
