#!/bin/bash
# the whole GPU suite and the bench on the current build
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5w}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_all.log" 2>&1 || { echo "ALL PYTEST FAILED"; tail -60 "$O/pytest_all.log"; exit 1; }
tail -1 "$O/pytest_all.log"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read())
x = d["extra"]
print(d["value"], d["kernels_us"], {k: x[k] for k in ("decode_1pct_loss", "two_stripes_two_streams", "host_batch_pipelined", "1000:1000x1024")})
PY
