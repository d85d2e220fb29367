#!/bin/bash
# Kernel trace of the 1000:1000 x 1 KiB codec (BASELINE configs[1]/[2]):
# bench line at that size, then rocprofv3 --kernel-trace of the same command
# (per-dispatch start / end: kernel durations and the gaps between them).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/small_${1:-x}"
mkdir -p "$O"
cd "$R"
B="--original 1000 --recovery 1000 --steps 50 --warmup 5 --no-cpu-baseline --no-extra"
timeout -k 10 120 python bench.py $B > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/bench.py" $B > "$O/trace.log" 2>&1
echo TRACE_DONE
