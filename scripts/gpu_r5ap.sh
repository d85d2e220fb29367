#!/bin/bash
# timing probe: the radix-2 column codec with every layer-0/1 twiddle load hitting one table (build_p, wrong results) vs build/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ap}"
mkdir -p "$O"
cd "$R"
for rep in 1 2 3; do
  for v in base p; do
    [ $v = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
    RS16_ROWS_NOCHECK=1 RS16_ROWS_ONLY=1000:1000,100:100,100:1000 RS16_LIB=$lib timeout -k 10 100 python -u scripts/reference_rows.py > "$O/rows_${v}_$rep.jsonl" 2>"$O/err" || { echo "ROWS FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $rep $(python3 -c "
import json
for l in open('$O/rows_${v}_$rep.jsonl'):
    d=json.loads(l); print(f\"{d['k']}:{d['m']} e{d['encode_us']} d1 {d['decode_1pct_us']} d100 {d['decode_100pct_us']}\", end=' | ')
")"
  done
done
