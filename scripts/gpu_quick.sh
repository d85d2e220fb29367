#!/bin/bash
# One gpurun call: GPU parity tests, then the bench (no CPU leg), each step
# with its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-q}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      ${PYTEST_ARGS:-} > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
