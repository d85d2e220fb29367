set -o pipefail
O=gpurun_out/r6sl2; mkdir -p $O
for r in 1 2 3; do
  for cfg in build:1 build:2 build_sq:2 build_s16:2 build_s16:1; do
    d=${cfg%%:*}; n=${cfg##*:}
    RS16_LIB=reed-solomon-16_amd/$d/librs16.so timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --slices $n > $O/${d}_s${n}_$r.json 2> $O/err.log || { echo FAIL $d $n; tail -20 $O/err.log; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d.get('kernels_us'))" $O/${d}_s${n}_$r.json $d $n
  done
done
