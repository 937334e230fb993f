set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3aa \
 "test|400|python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k 'sample or chunk_max or graph_replay or eos'" \
 "strace|200|python3 tools/sample_trace.py --model qwen2:1.5b" \
 "b1_q_cm|300|python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_q_old|300|CAIN_SAMPLE_CM=0 python3 bench.py --model qwen2:1.5b --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_l_cm|300|python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "b1_l_old|300|CAIN_SAMPLE_CM=0 python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy" \
 "prof_q|300|bash tools/prof_bench.sh r3aa/prof_b1_qwen2 --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-single --no-energy"
