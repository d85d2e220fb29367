#!/bin/bash
# r5l (host path + prepared tests, host batch probe, full bench), then a
# same-box A/B: base build, build_uni (timing-only upper bound: row 0's
# gather / reveal table for every row) and build_u2 (uniform-tile tables),
# then build_u2's decode parity tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5m}"
mkdir -p "$O"
cd "$R"
bash scripts/gpu_r5l.sh ${1:-r5m} || exit 1
for v in base uni u2 base uni u2; do
  [ "$v" = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --no-verify > "$O/ab_$v.json" 2>"$O/ab_err" || { echo "AB FAILED"; tail -20 "$O/ab_err"; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));k=d['kernels_us'];print(d['value'], round(sum(k.values()),1), k)")"
done
RS16_LIB=reed-solomon-16_amd/build_u2/librs16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_half_decode.py tests/test_gpu_device_path.py tests/test_gpu_batch.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/u2_pytest.log" 2>&1 || { echo "U2 PYTEST FAILED"; tail -40 "$O/u2_pytest.log"; exit 1; }
tail -1 "$O/u2_pytest.log"
