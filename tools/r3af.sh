set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r3af; mkdir -p $out/sq $out/tcc $out/attn
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/sq -o run -- python3 tools/wgemm_bench.py --no-lt --no-old --iters 10 --rows 256 > $out/sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/sq > $out/sq_summary.txt 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/tcc -o run -- python3 tools/wgemm_bench.py --no-lt --no-old --iters 10 --rows 256 > $out/tcc.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/tcc > $out/tcc_summary.txt 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/attn -o run -- python3 tools/bench_kernels.py --attn-only --attn 256:350,256:700,256:1400 > $out/attn.log 2>&1 || exit $?
python3 tools/pmc_summary.py $out/attn > $out/attn_summary.txt 2>&1
find $out -name "*.csv" -size +2M -delete
echo done
