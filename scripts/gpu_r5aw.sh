#!/bin/bash
# probe: ENC_MID at one workgroup per CU (build_p: 96 KiB of LDS, 2 dispatch rounds) vs build/, bench; then its stamps
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5aw}"
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for v in base p; do
    [ $v = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
    RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra > "$O/b_${v}_$rep.json" 2>"$O/err" || { echo "BENCH FAILED"; tail -20 "$O/err"; exit 1; }
    echo "$v $(python3 -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));k=d['kernels_us'];print(d['value'], k)")"
  done
done
RS16_LIB=reed-solomon-16_amd/build_ps/librs16.so RS16_STAMP_PROGS=ENC_MID RS16_STAMPS_OUT=stamps_probe1wg.json timeout -k 10 120 python -u scripts/stamps.py > "$O/st.log" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/st.log"; exit 1; }
cut -c1-900 "$O/st.log"
