#!/bin/bash
# ENC_MID over two items per workgroup (build_x) vs build/: parity on build_x, then bench A/B x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ax}"
mkdir -p "$O"
cd "$R"
RS16_LIB=reed-solomon-16_amd/build_x/librs16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_device_path.py tests/test_gpu_identity.py tests/test_gpu_half_decode.py tests/test_gpu_rate.py tests/test_gpu_fuzz.py tests/test_gpu_engine.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for rep in 1 2 3; do
  for v in base x; do
    [ $v = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_x/librs16.so
    RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra > "$O/b_${v}_$rep.json" 2>"$O/err" || { echo "BENCH FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $(python3 -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));k=d['kernels_us'];print(d['value'], round(sum(k.values()),1), k)")"
  done
done
