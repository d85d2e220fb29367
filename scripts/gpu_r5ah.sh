#!/bin/bash
# phase stamps of the column codec at 1000:1000 x 1 KiB: encode and the 1 %-loss general decode
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5ah}"
mkdir -p "$O"
cd "$R"
RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so RS16_STAMPS_LOSS=10 RS16_STAMP_PROGS=COL_ENC,COL_DEC RS16_STAMPS_OUT=stamps_col_1pct.json timeout -k 10 120 python -u scripts/stamps.py 1000 > "$O/st1.log" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/st1.log"; exit 1; }
cat "$O/st1.log" | cut -c1-900
