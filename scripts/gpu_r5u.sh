#!/bin/bash
# phase timeline of the 1 %-loss decode's kernels (stamps build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5u}"
mkdir -p "$O"
cd "$R"
RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so RS16_STAMPS_LOSS=327 RS16_STAMP_PROGS=DEC_MID_DIRECT RS16_STAMPS_OUT=r5u_stamps.json timeout -k 10 120 python -u scripts/stamps.py > "$O/stamps.log" 2>&1 || { echo "STAMPS FAILED"; tail -20 "$O/stamps.log"; exit 1; }
cat "$O/stamps.log"
timeout -k 10 120 python -u scripts/probe_1pct.py > "$O/p1.log" 2>&1 || { echo "P1 FAILED"; tail -20 "$O/p1.log"; exit 1; }
tail -3 "$O/p1.log" | head -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mid_direct.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_md.log" 2>&1 || { echo "MD PYTEST FAILED"; tail -60 "$O/pytest_md.log"; exit 1; }
tail -1 "$O/pytest_md.log"
