#!/bin/bash
# host batch rate vs lane stream priority (build_prio: greatest, build_lprio:
# least) and the number of streams created before the lanes
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5q}"
mkdir -p "$O"
cd "$R"
for v in prio lprio; do
  for pre in 0 1 2; do
    RS16_LIB=reed-solomon-16_amd/build_$v/librs16.so timeout -k 10 120 python -u scripts/probe_hostbatch.py 8 4 $pre > "$O/hb_${v}_$pre.log" 2>&1 || { echo "PROBE FAILED"; tail -20 "$O/hb_${v}_$pre.log"; exit 1; }
    echo "$v pre=$pre $(grep 'rep 3: encode' "$O/hb_${v}_$pre.log")"
  done
done
