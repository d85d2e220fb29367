#!/bin/bash
# One gpurun call: parity tests, bench, rocprofv3 kernel-trace stats, PMC
# passes (FETCH_SIZE / WRITE_SIZE / SQ groups, one per run), ablation builds
# and the microbenchmarks.  Every GPU step has its own time limit; the first
# failure ends the script.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-diag}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
fail() { echo "FAILED at $1"; tail -20 "$2" 2>/dev/null; exit 1; }
step() { echo "[$(date +%T)] $1"; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      > "$O/pytest.log" 2>&1 || fail pytest "$O/pytest.log"
  tail -1 "$O/pytest.log"
fi
step bench
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || fail bench "$O/bench.err"
cat "$O/bench.json"
if [ "${SKIP_UBENCH:-0}" != 1 ]; then
  for t in mem bfly valu; do
    step ubench_$t
    timeout -k 10 120 ./tools/ubench_$t > "$O/ubench_$t.txt" 2>&1 || fail ubench_$t "$O/ubench_$t.txt"
  done
fi
B="--steps 20 --warmup 5 --no-cpu-baseline --no-extra"
for v in ${VARIANTS-ab1 ab2 ab3 ab4}; do
  step "ablation $v"
  RS16_LIB="$R/reed-solomon-16_amd/build_$v/librs16.so" timeout -k 10 240 python bench.py $B --no-verify \
      > "$O/$v.json" 2> "$O/$v.err" || fail $v "$O/$v.err"
done
cd /tmp && export TMPDIR=/tmp
step rocprof-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" $B > "$O/bench_prof.log" 2>&1 || fail rocprof "$O/bench_prof.log"
P="--steps 5 --warmup 1 --no-cpu-baseline --no-extra"
i=0
for grp in FETCH_SIZE WRITE_SIZE \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
    ${EXTRA_PMC:-}; do
  i=$((i+1))
  step "pmc $i: $grp"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc$i" -o run --output-format csv \
      -- python3 "$R/bench.py" $P > "$O/pmc$i.log" 2>&1 || fail pmc$i "$O/pmc$i.log"
done
step done
