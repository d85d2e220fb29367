#!/bin/bash
# bench's host batch extra: main engine vs a fresh engine (RS16_BENCH_HB_ENGINE=fresh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5aa}"
mkdir -p "$O"
cd "$R"
for v in main fresh main fresh; do
  RS16_BENCH_HB_ENGINE=$v timeout -k 10 400 python bench.py --no-cpu-baseline > "$O/b_$v.json" 2>"$O/err" || { echo "BENCH FAILED"; tail -20 "$O/err"; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('$O/b_$v.json'));x=d['extra']['host_batch_pipelined'];print(d['value'], round(x['encode_gib_s'],1), round(x['decode_gib_s'],1))")"
done
