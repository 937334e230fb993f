set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3an \
 "l0|300|$B" \
 "l4|300|CAIN_SKINNY_W4=256 $B" \
 "l0b|300|$B" \
 "l4b|300|CAIN_SKINNY_W4=256 $B" \
 "m0|300|$B --model qwen2:7b" \
 "m4|300|CAIN_SKINNY_W4=256 $B --model qwen2:7b" \
 "prof|300|CAIN_SKINNY_W4=256 bash tools/prof_bench.sh r3an/prof_b1_llama_w4 --batch 1 --steps 1 --warmup 1 --no-single --no-energy"
