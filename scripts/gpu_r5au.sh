#!/bin/bash
# fused top layers of ENC_MID (build/) vs the previous commit (build_base/): parity, then bench A/B x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5au}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_path.py tests/test_gpu_rate.py tests/test_gpu_half_decode.py tests/test_gpu_identity.py tests/test_gpu_fuzz.py tests/test_gpu_batch.py tests/test_gpu_host_api.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for rep in 1 2 3; do
  for v in base x; do
    [ $v = x ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_base/librs16.so
    RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra > "$O/b_${v}_$rep.json" 2>"$O/err" || { echo "BENCH FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $(python3 -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));k=d['kernels_us'];print(d['value'], round(sum(k.values()),1), k)")"
  done
done
