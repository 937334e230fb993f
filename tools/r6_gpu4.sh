#!/usr/bin/env bash
# round 6: lean sampler as the default -- engine + sampler GPU tests, then the headline step with sampler mode 2
# (round-3 chunk-maximum kernel at 256 rows) vs 3 (lean), interleaved, then batch-1 on the seven models
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_lean_default; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sample_lean_gpu.py \
  tests/test_engine_gpu.py "tests/test_ops_gpu.py::test_sample_chunk_max_matches" \
  "tests/test_ops_gpu.py::test_sample_stop_ids_end_rows" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for mode in 2 3 2 3; do
  CAIN_SAMPLE_CM=$mode timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-single --no-energy \
    > $out/headline_cm$mode.json 2> $out/headline_cm$mode.err || { tail $out/headline_cm$mode.err; exit 1; }
  echo "cm$mode $(tail -1 $out/headline_cm$mode.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 600 python -u tools/b1_ab.py --dtype fp4 --trials 3 --label lean --out $out/b1_fp4.jsonl > /dev/null || exit 1
cat $out/b1_fp4.jsonl
