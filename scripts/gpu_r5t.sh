#!/bin/bash
# direct middle pass: timing-only variant without per-row LDS tables (build_mdx) vs this build
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5t}"
mkdir -p "$O"
cd "$R"
for v in new new; do
  [ "$v" = new ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -k 10 120 python -u scripts/probe_1pct.py > "$O/p1_$v.log" 2>&1 || { echo "P1 FAILED"; tail -20 "$O/p1_$v.log"; exit 1; }
  echo "$v $(tail -3 "$O/p1_$v.log" | head -1)"
done
