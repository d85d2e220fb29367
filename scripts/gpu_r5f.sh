#!/bin/bash
# GPU suite, stamps timelines of the 1 %-loss decodes (32768:32768 passes, 1000:1000 column codec), bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5f}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -60 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
export RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so
RS16_STAMPS_LOSS=327 RS16_STAMP_PROGS=EVAL_POLY,DEC_FIRST,DEC_MID,DEC_LAST RS16_STAMPS_OUT=${1:-r5f}/stamps_1pct.json \
  timeout -k 10 200 python scripts/stamps.py 32768 > "$O/stamps_1pct.txt" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/stamps_1pct.txt"; exit 1; }
RS16_STAMPS_LOSS=10 RS16_STAMP_PROGS=COL_DEC RS16_STAMPS_OUT=${1:-r5f}/stamps_col1pct.json \
  timeout -k 10 200 python scripts/stamps.py 1000 > "$O/stamps_col1pct.txt" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/stamps_col1pct.txt"; exit 1; }
RS16_STAMP_PROGS=COL_ENC,COL_DEC RS16_STAMPS_OUT=${1:-r5f}/stamps_col.json \
  timeout -k 10 200 python scripts/stamps.py 1000 > "$O/stamps_col.txt" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/stamps_col.txt"; exit 1; }
unset RS16_LIB
cut -c1-1200 "$O"/stamps_*.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read())
x = d["extra"]
print(d["value"], d["kernels_us"], "1pct", x["decode_1pct_loss"], "1000", x["1000:1000x1024"], "hostbatch", x["host_batch_pipelined"])
PY
