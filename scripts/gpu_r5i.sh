#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5i}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -60 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 200 python -u scripts/probe_hostbatch.py 8 6 > "$O/hb.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb.log"; exit 1; }
cat "$O/hb.log"
