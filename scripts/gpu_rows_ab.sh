#!/bin/bash
# Same-box A/B of library builds on the reference rows: parity of the first
# non-base variant (TESTS), then REPS rounds of scripts/reference_rows.py per
# variant (VARIANTS="base x y": base = build/, else build_<v>/).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-rows_ab}"
mkdir -p "$O"
cd "$R"
V=${VARIANTS:-base x}
first=$(echo $V | tr ' ' '\n' | grep -v '^base$' | head -1 || true)
if [ -n "$first" ] && [ -n "${TESTS:-}" ]; then
  RS16_LIB=reed-solomon-16_amd/build_$first/librs16.so timeout -k 10 500 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in $V; do
    [ $v = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
    RS16_LIB=$lib timeout -k 10 200 python -u scripts/reference_rows.py > "$O/rows_${v}_$rep.jsonl" 2>"$O/err" || { echo "ROWS FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $rep $(python3 -c "
import json
for l in open('$O/rows_${v}_$rep.jsonl'):
    d=json.loads(l)
    if d['k'] * d['m'] <= 1000000: print(f\"{d['k']}:{d['m']} e{d['encode_us']} d1 {d['decode_1pct_us']} d100 {d['decode_100pct_us']}\", end=' | ')
")"
  done
done
