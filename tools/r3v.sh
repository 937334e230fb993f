set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3v
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3v/bench_driver.log 2>&1 && \
bash tools/prof_bench.sh r3v/prof_head --steps 1 --warmup 1 --no-single --no-energy && \
bash tools/prof_bench.sh r3v/prof_b1_llama --batch 1 --steps 1 --warmup 1 --no-single --no-energy && \
bash tools/prof_bench.sh r3v/prof_b1_qwen2 --model qwen2:1.5b --batch 1 --steps 1 --warmup 1 --no-single --no-energy
