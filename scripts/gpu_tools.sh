#!/bin/bash
# One gpurun call: run prebuilt microbenchmark binaries under tools/ (names as
# arguments after the output tag), each under its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/$1"
shift
mkdir -p "$O"
cd "$R"
for t in "$@"; do
  timeout -k 10 120 "./tools/$t" > "$O/$t.txt" 2>&1 || { echo "$t FAILED"; cat "$O/$t.txt"; exit 1; }
  cat "$O/$t.txt"
done
