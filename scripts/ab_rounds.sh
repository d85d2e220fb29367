#!/bin/bash
# Same-box comparison of the round-5 final tree (exported to r5tree/ with its
# own bench.py and library: git archive e89d92f) against this tree:
# bench.py --no-extra --no-cpu-baseline, alternating, REPS times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r6rounds}"; mkdir -p "$O"
for r in $(seq 1 ${2:-5}); do
  (cd "$R/r5tree" && timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline > "$O/r5_$r.json" 2> "$O/err.log") || { echo FAIL r5; tail "$O/err.log"; exit 1; }
  (cd "$R" && timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline > "$O/r6_$r.json" 2> "$O/err.log") || { echo FAIL r6; tail "$O/err.log"; exit 1; }
  for t in r5 r6; do
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d.get('kernels_us'))" "$O/${t}_$r.json" $t $r
  done
done
