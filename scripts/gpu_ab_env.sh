#!/bin/bash
# Same-box A/B of environment settings: ENVS="A=1;B=2 ..." (space-separated
# variants, ';'-separated assignments; "-" = none) runs bench.py per variant.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abe
n=0
for v in ${ENVS:--}; do
  n=$((n+1))
  envs=""; [ "$v" != "-" ] && envs=$(echo "$v" | tr ';' ' ')
  env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS:-} > gpurun_out/abe/b_$n.json 2>gpurun_out/abe/err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/abe/b_$n.json'));k=d['kernels_us'];print(d['value'], round(sum(k.values()),1), k)")"
done
