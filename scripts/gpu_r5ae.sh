#!/bin/bash
# N = 2 rehearsal on one GPU (both ranks on GPU 0): the multi-rank bench path
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ae}"
mkdir -p "$O"
cd "$R"
RS16_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --no-cpu-baseline > "$O/bench_n2.json" 2> "$O/bench_n2.err" || { echo "BENCH N2 FAILED"; tail -30 "$O/bench_n2.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_n2.json'));print(d['value'], d['n_gpus'], d['ms_per_step'], sorted(d['extra'].keys()))"
