set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ab \
 "test|400|python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k 'sample or chunk_max or graph_replay or eos or wide_batch'" \
 "b_off|300|$B" \
 "b_cm|300|CAIN_SAMPLE_CM=2 $B" \
 "b_offb|300|$B" \
 "b_cmb|300|CAIN_SAMPLE_CM=2 $B" \
 "prof|300|CAIN_SAMPLE_CM=2 bash tools/prof_bench.sh r3ab/prof_head_cm --steps 1 --warmup 1 --no-single --no-energy"
