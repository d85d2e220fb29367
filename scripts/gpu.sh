#!/bin/bash
# One runner for every GPU job of this repo (run through gpurun from the repo
# root): a tag, then named steps run in order.  Each GPU step has its own
# time limit; the first failure ends the script (nothing more touches the GPU
# after a fault, an abort or a time limit).  Outputs go to gpurun_out/<tag>/.
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Steps:
#   tests[=PYTEST_ARGS]   pytest -m gpu (default: the whole suite under tests/)
#   bench[=ARGS]          python bench.py ARGS > bench.json (repeatable: bench_2.json, ...)
#   bench-n2[=ARGS]       the N = 2 driver launch with both ranks on GPU 0 (RS16_BENCH_SHARE_GPU=1)
#   stats[=ARGS]          rocprofv3 --kernel-trace --stats of bench.py ARGS (default: 20 steps, no extras)
#   pmc=COUNTERS[@SCRIPT] one rocprofv3 --pmc pass (counters comma-separated; default workload
#                         bench.py --steps 5 --no-extra, or SCRIPT with its arguments, '+' for spaces)
#   rows                  scripts/reference_rows.py > reference_rows.jsonl
#   probe=SCRIPT[+ARGS]   python scripts/SCRIPT ARGS ('+' separates arguments) > probe_N.log
#   tool=BINARY[+ARGS]    a tools/ microbenchmark
#   stamps=PROGS[+K]      phase timeline of pass programs PROGS (comma list) at k = m = K (default
#                         32768) with the stamps build (make -C reed-solomon-16_amd/csrc stamps:
#                         reed-solomon-16_amd/build_stamps/librs16.so) -> stamps_N.json
#   ab=DIRA,DIRB[+REPS[+ARGS]]  same-box A/B: bench.py --no-extra --no-cpu-baseline ARGS with
#                         RS16_LIB=reed-solomon-16_amd/DIRA/librs16.so, then DIRB, alternating, REPS (3) times
#   slices                bench.py at 1 / 2 / 4 column slices, fresh process per run, 3 reps
#                         (the profiles/r05_slices.txt measurement)
#
# Examples:
#   bash scripts/gpu.sh r06a tests bench stats
#   bash scripts/gpu.sh r06b 'tests=tests/test_gpu_prepared.py' 'probe=probe_1pct.py+5'
#   bash scripts/gpu.sh r06c 'pmc=FETCH_SIZE' 'pmc=WRITE_SIZE'
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
fail() { echo "FAILED at $1"; tail -30 "$2" 2>/dev/null; exit 1; }
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  case "$name" in
    tests)
      timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
          ${arg:-tests/} > "$O/pytest_$n.log" 2>&1 || fail tests "$O/pytest_$n.log"
      tail -1 "$O/pytest_$n.log" ;;
    bench)
      timeout -k 10 600 python bench.py $arg > "$O/bench_$n.json" 2> "$O/bench_$n.err" || fail bench "$O/bench_$n.err"
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('bench', d['value'], d['ms_per_step'], d.get('kernels_us'))" "$O/bench_$n.json" ;;
    bench-n2)
      RS16_BENCH_SHARE_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --no-cpu-baseline $arg > "$O/bench_n2_$n.json" \
          2> "$O/bench_n2_$n.err" || fail bench-n2 "$O/bench_n2_$n.err"
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('n2', d['value'], d['ms_per_step'], [(r['rank'], r['ms_per_step']) for r in d['ranks']])" "$O/bench_n2_$n.json" ;;
    stats)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/stats_$n" -o run \
          --output-format csv -- python3 "$R/bench.py" ${arg:---steps 20 --warmup 3 --no-cpu-baseline --no-extra} \
          > "$O/stats_$n.log" 2>&1) || fail stats "$O/stats_$n.log"
      echo "stats -> $O/stats_$n" ;;
    pmc)
      ctr=${arg%%@*}
      work="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra"
      [ "$ctr" != "$arg" ] && work="$R/scripts/${arg#*@}"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${ctr//,/ } \
          -d "$O/pmc_$n" -o run --output-format csv -- python3 ${work//+/ } > "$O/pmc_$n.log" 2>&1) \
          || fail pmc "$O/pmc_$n.log"
      echo "pmc $ctr -> $O/pmc_$n" ;;
    rows)
      timeout -k 10 300 python -u scripts/reference_rows.py > "$O/reference_rows.jsonl" 2> "$O/rows.err" \
          || fail rows "$O/rows.err"
      echo rows done ;;
    probe)
      timeout -k 10 500 python -u scripts/${arg//+/ } > "$O/probe_$n.log" 2>&1 || fail probe "$O/probe_$n.log"
      tail -40 "$O/probe_$n.log" ;;
    tool)
      timeout -k 10 120 ./tools/${arg//+/ } > "$O/tool_$n.log" 2>&1 || fail tool "$O/tool_$n.log"
      tail -40 "$O/tool_$n.log" ;;
    stamps)
      progs=${arg%%+*}
      size=""
      [ "$progs" != "$arg" ] && size=${arg#*+}
      RS16_LIB=reed-solomon-16_amd/build_stamps/librs16.so RS16_STAMP_PROGS=$progs RS16_STAMPS_OUT=$TAG/stamps_$n.json \
          timeout -k 10 300 python scripts/stamps.py $size > "$O/stamps_$n.txt" 2>&1 || fail stamps "$O/stamps_$n.txt"
      cut -c1-1500 "$O/stamps_$n.txt" ;;
    ab)
      dirs=${arg%%+*}
      rest=""
      [ "$dirs" != "$arg" ] && rest=${arg#*+}
      reps=${rest%%+*}
      bargs=""
      [ "$reps" != "$rest" ] && bargs=${rest#*+}
      for rep in $(seq 1 ${reps:-3}); do
        for d in ${dirs//,/ }; do
          RS16_LIB=reed-solomon-16_amd/$d/librs16.so timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline \
              ${bargs//+/ } > "$O/ab_${d}_$rep.json" 2> "$O/ab.err" || fail ab "$O/ab.err"
          echo "$d rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'], d['ms_per_step'], d['kernels_us'])" "$O/ab_${d}_$rep.json")"
        done
      done ;;
    slices)
      for rep in 1 2 3; do
        for sl in 1 2 4; do
          timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --slices $sl > "$O/sl_${sl}_$rep.json" \
              2> "$O/sl.err" || fail slices "$O/sl.err"
          echo "slices=$sl rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'], d['ms_per_step'])" "$O/sl_${sl}_$rep.json")"
        done
      done ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
done
echo "GPU_SH_DONE $TAG"
