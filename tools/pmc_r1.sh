#!/bin/bash
# PMC pass over the 128-row GEMM bodies (o: 4-wave narrow, gateup: 8-wave wide).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_r1 -o run -- python3 tools/bench_kernels.py --norm --rows 128 --roles o,gateup --gemm-only > gpurun_out/pmc_r1/bench.log 2>&1
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc_r1 > gpurun_out/pmc_r1/summary.txt 2>&1
find gpurun_out/pmc_r1 -name "*.csv" -size +2M -delete
cat gpurun_out/pmc_r1/summary.txt | head -60
exit $rc
