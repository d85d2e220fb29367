#!/bin/bash
# host batch lanes after an RCCL communicator / after the one-shot host path (as bench.py runs them)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5z}"
mkdir -p "$O"
cd "$R"
for mode in rccl rccl rccl oneshot oneshot oneshot; do
  timeout -k 10 120 python -u scripts/probe_hostbatch.py 8 4 0 $mode > "$O/hb.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb.log"; exit 1; }
  echo "$mode $(grep 'rep 3: encode' "$O/hb.log")"
done
