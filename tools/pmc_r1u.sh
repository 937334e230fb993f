#!/bin/bash
# PMC pass over the 256-row GEMM bodies (o, gateup, down).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r1u
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_r1u -o run -- python3 tools/bench_kernels.py --norm --rows 256 --roles o,gateup,down --gemm-only > gpurun_out/pmc_r1u/bench.log 2>&1
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc_r1u > gpurun_out/pmc_r1u/summary.txt 2>&1
find gpurun_out/pmc_r1u -name "*.csv" -size +2M -delete
cat gpurun_out/pmc_r1u/summary.txt | head -60
exit $rc
