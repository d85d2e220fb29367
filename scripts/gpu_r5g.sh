#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5g}"
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python -u scripts/probe_hostbatch.py > "$O/hostbatch.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hostbatch.log"; exit 1; }
cat "$O/hostbatch.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/prof" -o hb -- python3 "$R/scripts/probe_hostbatch.py" 4 > "$O/prof.log" 2>&1 || { echo "PROF FAILED"; tail -20 "$O/prof.log"; exit 1; }
find "$O/prof" -name "*.csv" | head
