#!/bin/bash
# One gpurun call: the VALU issue-rate microbenchmarks (tools/ubench_valu,
# tools/ubench_bfly, built here beforehand), then the bench without extras.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-ubench}"
mkdir -p "$O"
cd "$R"
timeout -k 10 120 ./tools/ubench_valu > "$O/ubench_valu.txt" 2>&1 || { echo "UBENCH_VALU FAILED"; cat "$O/ubench_valu.txt"; exit 1; }
timeout -k 10 120 ./tools/ubench_bfly > "$O/ubench_bfly.txt" 2>&1 || { echo "UBENCH_BFLY FAILED"; cat "$O/ubench_bfly.txt"; exit 1; }
cat "$O/ubench_valu.txt" "$O/ubench_bfly.txt"
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { echo "BENCH FAILED"; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
