set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgemm_gpu.py > gpurun_out/r6w/wgemm_tests.log 2>&1 || { tail -30 gpurun_out/r6w/wgemm_tests.log; exit 1; }
tail -2 gpurun_out/r6w/wgemm_tests.log
for i in 1 2; do
  for m in 0 1; do
    CAIN_WGEMM_INLINE=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-single > gpurun_out/r6w/bench_inl${m}_$i.json 2> gpurun_out/r6w/bench_inl${m}_$i.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/r6w/bench_inl${m}_$i.json').read().strip().splitlines()[-1]);print('inline=$m', d['value'], d['J_per_token'], d['ms_per_step'])"
  done
done
