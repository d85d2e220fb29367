#!/bin/bash
# HW queue experiment: the queue probe and the bench with 16 hardware queues per process vs the default (4).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5e}"
mkdir -p "$O"
cd "$R"
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u scripts/probe_queues.py > "$O/queues16.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/queues16.log"; exit 1; }
tail -1 "$O/queues16.log"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$O/bench_q4.json" 2> "$O/bench_q4.err" || { echo "BENCH FAILED"; tail -20 "$O/bench_q4.err"; exit 1; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python bench.py --no-cpu-baseline > "$O/bench_q16.json" 2> "$O/bench_q16.err" || { echo "BENCH FAILED"; tail -20 "$O/bench_q16.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
for f in ("bench_q4.json", "bench_q16.json"):
    d = json.loads(open(sys.argv[1] + "/" + f).read())
    x = d["extra"]
    print(f, d["value"], d["kernels_us"], "sustained", x["sustained"]["gib_s"], "two", x["two_stripes_two_streams"]["gib_s"],
          x["two_stripes_two_streams"]["right_after_timed_loop"]["gib_s"], "encdec",
          x["two_stripes_two_streams"]["encode_while_decode_gib_s"], "1pct", x["decode_1pct_loss"]["decode_gib_s"],
          "hostbatch", x["host_batch_pipelined"]["encode_gib_s"], x["host_batch_pipelined"]["decode_gib_s"])
PY
