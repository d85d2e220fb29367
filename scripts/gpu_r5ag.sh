#!/bin/bash
# column general decode with zero-block / no-output wave skipping (build_x) vs build/: parity, then reference rows x2 each
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ag}"
mkdir -p "$O"
cd "$R"
RS16_LIB=reed-solomon-16_amd/build_x/librs16.so timeout -k 10 500 python -u -m pytest tests/test_gpu_col.py tests/test_gpu_fuzz.py tests/test_gpu_rate.py tests/test_gpu_host_api.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/x_pytest.log" 2>&1 || { echo "X PYTEST FAILED"; tail -40 "$O/x_pytest.log"; exit 1; }
tail -1 "$O/x_pytest.log"
for rep in 1 2; do
  for v in base x; do
    [ $v = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_x/librs16.so
    RS16_LIB=$lib timeout -k 10 200 python -u scripts/reference_rows.py > "$O/rows_${v}_$rep.jsonl" 2>"$O/err" || { echo "ROWS FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $rep $(python3 -c "
import json
for l in open('$O/rows_${v}_$rep.jsonl'):
    d=json.loads(l); print(f\"{d['k']}:{d['m']} e{d['encode_us']} d1 {d['decode_1pct_us']} d100 {d['decode_100pct_us']}\", end=' | ')
")"
  done
done
