#!/bin/bash
# Column codec: GPU tests, probe, stamps timeline (stamps build), optional full suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-col}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
bash scripts/gpu_col.sh "$TAG" || exit 1
RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so RS16_STAMP_PROGS=COL_ENC,COL_DEC RS16_STAMPS_OUT=$TAG/stamps.json \
  timeout -k 10 200 python scripts/stamps.py 1000 > "$O/stamps.txt" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/stamps.txt"; exit 1; }
cut -c1-900 "$O/stamps.txt"
