set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3aq \
 "gputest|900|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke|200|python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
