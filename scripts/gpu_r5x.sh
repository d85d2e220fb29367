#!/bin/bash
# host-link copies: copy engines vs copy kernels (tools/ubench_pcie.hip)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-r5x}"
mkdir -p "$O"
cd "$R"
for b in 64 256 1024; do
  echo "== blocks $b"
  timeout -k 10 60 ./tools/ubench_pcie $b || { echo "UBENCH FAILED"; exit 1; }
done
