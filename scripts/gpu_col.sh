#!/bin/bash
# One gpurun call: the column-codec GPU tests, the column-vs-pass probe, then
# (optionally) the whole GPU suite; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-col}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_col.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest_col.log" 2>&1 || { echo "COL TESTS FAILED"; tail -40 "$O/pytest_col.log"; exit 1; }
tail -1 "$O/pytest_col.log"
timeout -k 10 300 python -u scripts/probe_col.py > "$O/probe.jsonl" 2> "$O/probe.err" || { echo "PROBE FAILED"; tail -20 "$O/probe.err"; exit 1; }
cat "$O/probe.jsonl"
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
