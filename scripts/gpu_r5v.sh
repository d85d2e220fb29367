#!/bin/bash
# the bench step with 1 / 2 / 4 column slices on forked streams (fresh process each)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5v}"
mkdir -p "$O"
cd "$R"
for rep in 1 2 3; do
  for sl in 1 2 4; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --slices $sl > "$O/b_${sl}_$rep.json" 2>"$O/err" || { echo "BENCH FAILED"; tail -20 "$O/err"; exit 1; }
    echo "slices=$sl rep=$rep $(python3 -c "import json;d=json.load(open('$O/b_${sl}_$rep.json'));print(d['value'], d['ms_per_step'])")"
  done
done
