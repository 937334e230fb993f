#!/bin/bash
# PMC pass over the wide GEMM (tools/wgemm_bench.py) -> gpurun_out/<tag>/summary.txt
# usage: tools/pmc_wgemm.sh <tag> <wgemm_bench args...>
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out -o run -- python3 tools/wgemm_bench.py --no-lt --no-old --iters 10 "$@" > $out/bench.log 2>&1
rc=$?
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
find $out -name "*.csv" -size +2M -delete
exit $rc
