#!/bin/bash
# host-link rates against the NUMA node the process is bound to
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ab}"
mkdir -p "$O"
cd "$R"
for n in 0 1 0 1; do
  timeout -k 10 120 python -u scripts/probe_numa.py $n 2>&1 | tail -4 || { echo "PROBE FAILED"; exit 1; }
done
