#!/bin/bash
# identity-multiplier decode: its tests, the whole GPU suite, then a same-box
# A/B against the previous build (build_base) and the full bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5n}"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_identity.py tests/test_gpu_half_decode.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_id.log" 2>&1 || { echo "ID PYTEST FAILED"; tail -60 "$O/pytest_id.log"; exit 1; }
tail -1 "$O/pytest_id.log"
for v in base new base new; do
  [ "$v" = new ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra > "$O/ab_$v.json" 2>"$O/ab_err" || { echo "AB FAILED"; tail -20 "$O/ab_err"; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));k=d['kernels_us'];print(d['value'], d['ms_per_step'], round(sum(k.values()),1), k)")"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_all.log" 2>&1 || { echo "ALL PYTEST FAILED"; tail -60 "$O/pytest_all.log"; exit 1; }
tail -1 "$O/pytest_all.log"
