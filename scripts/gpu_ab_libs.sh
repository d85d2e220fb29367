#!/bin/bash
# Same-box A/B of library builds: VARIANTS="base x y ..." runs bench.py with
# RS16_LIB=reed-solomon-16_amd/build_<v>/librs16.so (base = build/) and
# prints the value and the per-pass hipEvent times of each run.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
n=0
for v in ${VARIANTS:-base}; do
  n=$((n+1))
  [ "$v" = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS:-} > gpurun_out/ab/b_${n}_$v.json 2>gpurun_out/ab/err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab/b_${n}_$v.json'));k=d['kernels_us'];print(d['value'], round(sum(k.values()),1), k)")"
done
