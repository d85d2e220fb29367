#!/bin/bash
# One gpurun call for the column codec round: column tests + probe, the
# whole GPU suite, smoke, the bench line, the rocprofv3 kernel-trace stats
# of the bench and of the 1000:1000 codec.  First failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3b}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
FULL=1 bash scripts/gpu_col.sh "$TAG" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "SMOKE FAILED"; tail -20 "$O/smoke.log"; exit 1; }
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
cut -c1-400 "$O/bench.json"
bash scripts/gpu_small_trace.sh "$TAG" > "$O/small.log" 2>&1 || { echo "SMALL TRACE FAILED"; tail -20 "$O/small.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extra > "$O/bench_prof.json" 2> "$O/bench_prof.err" \
    || { echo "PROF FAILED"; tail -20 "$O/bench_prof.err"; exit 1; }
echo ROUND_DONE
