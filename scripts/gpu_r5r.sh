#!/bin/bash
# direct middle pass: its tests and the GPU suite's decode tests, the 1 %
# decode timing (base build vs this build), host batch lanes with CU-masked
# streams (build_cum)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5r}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mid_direct.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_md.log" 2>&1 || { echo "MD PYTEST FAILED"; tail -60 "$O/pytest_md.log"; exit 1; }
tail -1 "$O/pytest_md.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_path.py tests/test_gpu_fuzz.py tests/test_gpu_batch.py tests/test_gpu_rate.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_dec.log" 2>&1 || { echo "DEC PYTEST FAILED"; tail -60 "$O/pytest_dec.log"; exit 1; }
tail -1 "$O/pytest_dec.log"
for v in base new base new; do
  [ "$v" = new ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -k 10 120 python -u scripts/probe_1pct.py > "$O/p1_$v.log" 2>&1 || { echo "P1 FAILED"; tail -20 "$O/p1_$v.log"; exit 1; }
  echo "$v $(tail -3 "$O/p1_$v.log" | tr '\n' ' ')"
done
for pre in 0 1 2; do
  RS16_LIB=reed-solomon-16_amd/build_cum/librs16.so timeout -k 10 120 python -u scripts/probe_hostbatch.py 8 4 $pre > "$O/hb_cum_$pre.log" 2>&1 || { echo "HB FAILED"; tail -20 "$O/hb_cum_$pre.log"; exit 1; }
  echo "cum pre=$pre $(grep 'rep 3: encode' "$O/hb_cum_$pre.log")"
done
