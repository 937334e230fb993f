#!/usr/bin/env bash
# PMC counters of the batch-1 gate/up GEMM: MXFP4 (gemm_w4.hip) vs GGUF Q4_0 (gemm_q4.hip), kernel trace + stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6pmc
for dt in fp4 q4_0; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --stats -d gpurun_out/r6pmc/$dt -o pmc -- python3 tools/w4_bench.py --roles gateup --dtypes $dt --variants rule > gpurun_out/r6pmc/$dt.log 2>&1 || exit 1
done
