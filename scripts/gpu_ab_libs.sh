set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-"" st1 st2}; do
  [ "$v" = base ] && lib=reed-solomon-16_amd/build/librs16.so || lib=reed-solomon-16_amd/build${v:+_$v}/librs16.so
  RS16_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra > gpurun_out/ab/b_${v:-base}.json 2>gpurun_out/ab/err
  echo "${v:-base} $(python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/b_${v:-base}.json'));print(d['value'], d.get('kernels_us'))")"
done
