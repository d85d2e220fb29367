#!/bin/bash
# rocprofv3 PMC passes (one counter group per run; --kernel-trace/--stats only).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dev}
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-extra ${EXTRA_ARGS:-}"
if [ "${LIST:-0}" = "1" ]; then rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true; fi
i=0
for grp in "${@:2}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
done
echo PMC_DONE
