#!/bin/bash
# Round 5: GPU suite (with the widened fuzzer, timed), then the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5b}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    --durations=15 ${PYTEST_ARGS:-} > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -60 "$O/pytest.log"; exit 1; }
tail -25 "$O/pytest.log"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
