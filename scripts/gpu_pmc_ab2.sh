set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pab
cd /tmp && export TMPDIR=/tmp
for v in ab5 base; do
  [ "$v" = base ] && lib=$R/reed-solomon-16_amd/build/librs16.so || lib=$R/reed-solomon-16_amd/build_$v/librs16.so
  RS16_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $R/gpurun_out/pab/$v -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra --no-verify > $R/gpurun_out/pab/$v.log 2>&1
  python3 $R/scripts/pmc_summary.py $R/gpurun_out/pab/$v/run_counter_collection.csv | cut -c1-200
done
