set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
F="python3 bench.py --batch 1 --weights fp8 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3aj \
 "test|300|python -u -m pytest tests/test_w8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "test8|300|CAIN_W8_U=8 python -u -m pytest tests/test_w8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "testb|300|CAIN_SKINNY_XLDS=8 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k skinny" \
 "f_def|300|$F" \
 "f_u8|300|CAIN_W8_U=8 $F" \
 "f_u4w8|300|CAIN_W8_WAVES=8 $F" \
 "f_def_b|300|$F" \
 "f_u8_b|300|CAIN_W8_U=8 $F" \
 "fq_def|300|$F --model qwen2:1.5b" \
 "fq_u8|300|CAIN_W8_U=8 $F --model qwen2:1.5b" \
 "l0|300|$B" \
 "l8|300|CAIN_SKINNY_XLDS=8 $B" \
 "q0|300|$B --model qwen2:1.5b" \
 "q8|300|CAIN_SKINNY_XLDS=8 $B --model qwen2:1.5b" \
 "prof|300|bash tools/prof_bench.sh r3aj/prof_b1_llama_fp8_xl_u4 --batch 1 --weights fp8 --steps 1 --warmup 1 --no-single --no-energy"
