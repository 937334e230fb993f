#!/bin/bash
# After full-line staging: ring depth / k-split / waves at 128 rows; PMC pass on o and gateup.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/sweep_r1e.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_D=0 || exit 1
run CAIN_BGEMM_D=4 || exit 1
run CAIN_BGEMM_D=6 || exit 1
run CAIN_BGEMM_D=8 || exit 1
run CAIN_BGEMM_WG=256 || exit 1
run CAIN_BGEMM_WG=512 || exit 1
run CAIN_BGEMM_W=8 || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r1e
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_r1e -o run -- python3 tools/bench_kernels.py --norm --rows 128 --roles o,gateup --gemm-only > gpurun_out/pmc_r1e/bench.log 2>&1
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc_r1e > gpurun_out/pmc_r1e/summary.txt 2>&1
find gpurun_out/pmc_r1e -name "*.csv" -size +2M -delete
grep -A 10 bgemm gpurun_out/pmc_r1e/summary.txt
exit $rc
