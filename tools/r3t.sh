set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3t \
 "gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'"
