#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5l}"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_prepared.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -60 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 200 python -u scripts/probe_hostbatch.py 8 5 > "$O/hb.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb.log"; exit 1; }
cat "$O/hb.log"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read())
x = d["extra"]
print(d["value"], d["kernels_us"], {k: x[k] for k in ("split_decode_step", "two_stripes_two_streams", "host_batch_pipelined", "host_resident_pcie", "decode_1pct_loss", "1000:1000x1024")})
PY
