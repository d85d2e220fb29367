#!/bin/bash
# Same-box A/B of environment settings of the pass kernels (experiment knobs):
# bench.py (no extras, 200 steps) once per setting per round, alternating.
# usage: bash scripts/ab_env_bench.sh ROUNDS "ENV1" "ENV2" ...   (ENV "-" = none)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
rounds=$1; shift
for i in $(seq 1 "$rounds"); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then envs=(); else read -ra envs <<< "$e"; fi
    out=$(env "${envs[@]}" timeout -k 10 120 python bench.py --steps 200 --warmup 50 --no-extra --no-cpu-baseline) || { echo "FAILED $e"; exit 1; }
    python3 -c "
import json,sys
d=json.loads(sys.argv[2].strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], json.dumps(d.get('kernels_us')))" "$e" "$out"
  done
done
