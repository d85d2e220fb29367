#!/bin/bash
# Round 5: the GPU suite, then the two-stripe reconciliation probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5a}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS:-} > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -u scripts/probe_reconcile.py > "$O/reconcile.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/reconcile.log"; exit 1; }
cat "$O/reconcile.log"
