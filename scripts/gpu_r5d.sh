#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5d}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u scripts/probe_queues.py > "$O/queues.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/queues.log"; exit 1; }
cat "$O/queues.log"
