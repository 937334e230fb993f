set -o pipefail
export TMPDIR=/tmp
F="python3 bench.py --batch 1 --weights fp8 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3al \
 "test|300|python -u -m pytest tests/test_w8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "f_new|300|$F" \
 "f_old|300|CAIN_W8_WAVE_BOUND=511 $F" \
 "f_new_b|300|$F" \
 "f_old_b|300|CAIN_W8_WAVE_BOUND=511 $F" \
 "fq|300|$F --model qwen2:1.5b" \
 "fm|300|$F --model mistral:7b" \
 "fq7|300|$F --model qwen2:7b" \
 "fq7o|300|CAIN_W8_WAVE_BOUND=511 $F --model qwen2:7b" \
 "prof|300|bash tools/prof_bench.sh r3al/prof_b1_llama_fp8_final --batch 1 --weights fp8 --steps 1 --warmup 1 --no-single --no-energy"
