#!/bin/bash
# Shipped build vs diagnostic variants (RS16_ABLATE=1: no butterfly layers;
# =2: no HBM loads/stores; build_np: no register pins).
set -e
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --no-cpu-baseline --no-extra"
timeout -k 10 240 python bench.py $B > gpurun_out/ab0.json
for v in ${VARIANTS:-ab1 ab2}; do
  RS16_LIB=reed-solomon-16_amd/build_$v/librs16.so timeout -k 10 240 python bench.py $B --no-verify > gpurun_out/$v.json
done
echo done
