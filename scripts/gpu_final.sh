#!/bin/bash
# End-of-round measurement on one box (run via gpurun): the GPU test suite,
# the bench line, the round profile (rocprof stats + PMC passes,
# scripts/gpu_profile.sh) and the reference benchmark rows.  Every GPU step
# has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
O="$R/gpurun_out/final_$TAG"
mkdir -p "$O"
cd "$R"
fail() { echo "FAILED at $1"; tail -20 "$2" 2>/dev/null; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > "$O/pytest.log" 2>&1 || fail pytest "$O/pytest.log"
tail -1 "$O/pytest.log"
timeout -k 10 300 python -u scripts/reference_rows.py > "$O/reference_rows.jsonl" 2> "$O/reference_rows.err" || fail rows "$O/reference_rows.err"
echo rows done
bash scripts/gpu_profile.sh "$TAG" > "$O/profile.log" 2>&1 || fail profile "$O/profile.log"
echo FINAL_DONE
