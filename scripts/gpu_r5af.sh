#!/bin/bash
# early stores of the IFFT-only passes (build_x) vs without (build_base): parity, then A/B x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5af}"
mkdir -p "$O"
cd "$R"
RS16_LIB=reed-solomon-16_amd/build_x/librs16.so timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_engine.py tests/test_gpu_identity.py tests/test_gpu_device_path.py tests/test_gpu_half_decode.py tests/test_gpu_batch.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/x_pytest.log" 2>&1 || { echo "X PYTEST FAILED"; tail -40 "$O/x_pytest.log"; exit 1; }
tail -1 "$O/x_pytest.log"
for rep in 1 2 3; do
  for v in base x; do
    RS16_LIB=reed-solomon-16_amd/build_$v/librs16.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra > "$O/b_${v}_$rep.json" 2>"$O/err" || { echo "BENCH FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $(python3 -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));k=d['kernels_us'];print(d['value'], round(sum(k.values()),1), k)")"
  done
done
