#!/bin/bash
# host batch lanes: rate against streams created before them, fresh process each
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5y}"
mkdir -p "$O"
cd "$R"
for pre in 0 0 0 5 10 20 20; do
  timeout -k 10 120 python -u scripts/probe_hostbatch.py 8 4 $pre > "$O/hb.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb.log"; exit 1; }
  echo "pre=$pre $(grep 'rep 3: encode' "$O/hb.log")"
done
