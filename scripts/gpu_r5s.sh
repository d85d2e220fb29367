#!/bin/bash
# direct middle pass, 8-wave form: its tests, the 1 % decode timing
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5s}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mid_direct.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_md.log" 2>&1 || { echo "MD PYTEST FAILED"; tail -60 "$O/pytest_md.log"; exit 1; }
tail -1 "$O/pytest_md.log"
for v in new new; do
  timeout -k 10 120 python -u scripts/probe_1pct.py > "$O/p1_$v.log" 2>&1 || { echo "P1 FAILED"; tail -20 "$O/p1_$v.log"; exit 1; }
  echo "$v $(tail -3 "$O/p1_$v.log" | head -1)"
done
