#!/bin/bash
# One gpurun call: GPU tests, smoke, the full bench line, and the rocprofv3
# kernel-trace summary of a short bench run; each step under its own limit,
# the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "SMOKE FAILED"; tail -20 "$O/smoke.log"; exit 1; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extra > "$O/bench_prof.json" 2> "$O/bench_prof.err" \
    || { echo "PROF FAILED"; tail -20 "$O/bench_prof.err"; exit 1; }
echo ROUND_DONE
