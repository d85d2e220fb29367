#!/bin/bash
# GPU parity tests, then a quick bench (run via gpurun).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dev}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout=300 > gpurun_out/pytest_$TAG.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
tail -1 gpurun_out/bench_$TAG.log
