#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5h}"
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python -u scripts/probe_hostbatch.py 8 6 > "$O/hb_sdma.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb_sdma.log"; exit 1; }
cat "$O/hb_sdma.log"
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u scripts/probe_hostbatch.py 8 6 > "$O/hb_blit.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb_blit.log"; exit 1; }
cat "$O/hb_blit.log"
