#!/bin/bash
# Round profile (run via gpurun): bench line, rocprofv3 kernel-trace stats of
# the same bench command, PMC FETCH_SIZE / WRITE_SIZE passes (one group per
# run) and two SQ counter groups.  Every GPU step has its own time limit;
# the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
O="$R/gpurun_out/prof_$TAG"
mkdir -p "$O"
cd "$R"
fail() { echo "FAILED at $1"; tail -20 "$2" 2>/dev/null; exit 1; }
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || fail bench "$O/bench.err"
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
B="--steps 20 --warmup 3 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv \
    -- python3 "$R/bench.py" $B > "$O/stats.log" 2>&1 || fail stats "$O/stats.log"
P="--steps 5 --warmup 1 --no-cpu-baseline --no-extra"
i=0
for grp in FETCH_SIZE WRITE_SIZE \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc$i" -o run --output-format csv \
      -- python3 "$R/bench.py" $P > "$O/pmc$i.log" 2>&1 || fail pmc$i "$O/pmc$i.log"
done
# the same traffic counters over the 1 %-loss general decode and the column
# codec's 1000:1000 workloads (scripts/pmc_extra.py)
for grp in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$O/pmc$i" -o run --output-format csv \
      -- python3 "$R/scripts/pmc_extra.py" 5 > "$O/pmc$i.log" 2>&1 || fail pmc$i "$O/pmc$i.log"
done
echo PROFILE_DONE
