#!/bin/bash
# Which earlier bench extra slows the in-process pipelined host batch (VERDICT
# r5 item 4)?  bench.py --no-cpu-baseline with every extra but the host batch
# and one candidate skipped (RS16_BENCH_SKIP), then with all of them.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-hb_bisect}"
mkdir -p "$O"
cd "$R"
ALL="two_stripes sustained kib1000 decode_1pct general_decodes rate_paths configs4 host_resident api_loop"
for keep in none configs4 rate_paths kib1000 two_stripes general_decodes host_resident all; do
  skip=""
  for x in $ALL; do [ "$x" != "$keep" ] && [ "$keep" != all ] && skip="$skip,$x"; done
  RS16_BENCH_SKIP=${skip#,} timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/b_$keep.json" 2> "$O/b_$keep.err" \
      || { echo "BENCH FAILED ($keep)"; tail -20 "$O/b_$keep.err"; exit 1; }
  echo "keep=$keep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));x=d['extra'].get('host_batch_pipelined',{});f=x.get('fresh_process',{});print(d['value'], round(x.get('encode_gib_s',0),1), round(x.get('decode_gib_s',0),1), 'fresh', f.get('encode_gib_s'), f.get('decode_gib_s'))" "$O/b_$keep.json")"
done
