#!/bin/bash
# smoke + bench + rocprofv3 kernel-trace stats on one MI355X (run via gpurun).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extra > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
echo DONE
