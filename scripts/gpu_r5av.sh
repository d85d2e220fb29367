#!/bin/bash
# phase stamps of the bench step's passes (32768:32768 x 1 KiB, encode + identity half decode)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5av}"
mkdir -p "$O"
cd "$R"
RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so RS16_STAMP_PROGS=ENC_FIRST,ENC_MID,ENC_LAST RS16_STAMPS_OUT=stamps_passes.json timeout -k 10 120 python -u scripts/stamps.py > "$O/st.log" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/st.log"; exit 1; }
cut -c1-700 "$O/st.log"
