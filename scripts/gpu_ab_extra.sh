#!/bin/bash
# Same-box A/B of library builds on bench.py's extras: VARIANTS="base x ..."
# (base = build/, x = build_x/), KEYS = the extra entries to print.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abx
n=0
for v in ${VARIANTS:-base}; do
  n=$((n+1))
  [ "$v" = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abx/b_${n}_$v.json 2>gpurun_out/abx/err_$n
  echo "$v $(python3 -c "
import json,sys
d=json.load(open('gpurun_out/abx/b_${n}_$v.json'))
print(d['value'], {k: d['extra'].get(k) for k in '${KEYS:-rate_paths}'.split(',')})")"
done
