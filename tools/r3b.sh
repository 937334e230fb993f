set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_continuous_gpu.py tests/test_lt_gpu.py tests/test_wgemm_gpu.py tests/test_study.py -m gpu > gpurun_out/r3b/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3b/pytest.log; exit $rc
