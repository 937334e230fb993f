set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3x
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3x/bench_driver.log 2>&1 || exit $?
for m in qwen2:1.5b gemma:2b phi3:3.8b qwen2:7b mistral:7b gemma:7b llama3.1:8b; do
  timeout -k 10 300 python3 bench.py --model $m --words 1000 --steps 2 --warmup 1 --no-single > "gpurun_out/r3x/model_${m}.log" 2>&1 || exit $?
done
