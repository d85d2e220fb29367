#!/bin/bash
# Round-6 measurement set on one box: the bench line (python bench.py), the
# rocprofv3 kernel-trace summary of the same command, the reference rows, a
# memory-copy trace of tools/ubench_pcie (copy-engine pairs).  Every GPU step
# has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
O="$R/gpurun_out/final_$TAG"
mkdir -p "$O"
cd "$R"
fail() { echo "FAILED at $1"; tail -20 "$2" 2>/dev/null; exit 1; }
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || fail bench "$O/bench.err"
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['kernels_us'])"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extra \
    > "$O/stats.log" 2>&1) || fail stats "$O/stats.log"
echo stats done
timeout -k 10 300 python -u scripts/reference_rows.py > "$O/reference_rows.jsonl" 2> "$O/rows.err" || fail rows "$O/rows.err"
echo rows done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --memory-copy-trace -d "$O/pcie_tr" -o run \
    --output-format csv -- "$R/tools/ubench_pcie" 64 > "$O/pcie_tr.log" 2>&1) || fail pcie "$O/pcie_tr.log"
head -4 "$O/pcie_tr.log"
echo ROUND6_DONE
