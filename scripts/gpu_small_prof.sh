#!/bin/bash
# Kernel-trace stats of the 1000:1000 x 1 KiB configuration (BASELINE
# configs[1] / [2]): bench line at that size, then rocprofv3 --stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-small}
O="$R/gpurun_out/prof_$TAG"
mkdir -p "$O"
cd "$R"
B="--original 1000 --recovery 1000 --steps 200 --warmup 20 --no-cpu-baseline --no-extra"
timeout -k 10 300 python bench.py $B > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv \
    -- python3 "$R/bench.py" $B > "$O/stats.log" 2>&1 || { tail -20 "$O/stats.log"; exit 1; }
find "$O/stats" -name '*kernel_stats.csv' -exec cut -c1-150 {} \;
