#!/bin/bash
# host batch right after seconds of device-resident steps
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ac}"
mkdir -p "$O"
cd "$R"
for mode in hot3 hot3 cold hot10; do
  timeout -k 10 120 python -u scripts/probe_hostbatch.py 8 4 0 $mode > "$O/hb.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb.log"; exit 1; }
  echo "$mode $(grep 'rep 0: encode' "$O/hb.log") | $(grep 'rep 3: encode' "$O/hb.log") | $(grep 'rep 3: one-shot' "$O/hb.log")"
done
