#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5c}"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u scripts/probe_reconcile2.py > "$O/reconcile2.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/reconcile2.log"; exit 1; }
cat "$O/reconcile2.log"
