#!/bin/bash
# host batch rate against the number of streams created before its lanes
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5p}"
mkdir -p "$O"
cd "$R"
for pre in 0 1 2 3; do
  timeout -k 10 120 python -u scripts/probe_hostbatch.py 8 4 $pre > "$O/hb_$pre.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb_$pre.log"; exit 1; }
  grep "rep 3" "$O/hb_$pre.log"
done
