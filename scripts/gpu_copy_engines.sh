#!/bin/bash
# Which SDMA engine does the HIP runtime give each copy?  tools/ubench_pcie in
# fresh processes with the runtime's copy log on (AMD_LOG_LEVEL=4): its
# "Query copy engine status" (free / recommended engine masks) and "HSA Copy
# copy_engine=" lines, beside the pair rates of the same process.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-copy_engines}"
mkdir -p "$O"
cd "$R"
for i in 1 2 3 4; do
  AMD_LOG_LEVEL=4 timeout -k 10 120 ./tools/ubench_pcie 64 > "$O/pcie_$i.txt" 2> "$O/pcie_$i.log" || { echo "UBENCH FAILED"; tail "$O/pcie_$i.log"; exit 1; }
  echo "== process $i: $(grep "cpu " "$O/pcie_$i.txt") $(grep "H2D + D2H on two streams" "$O/pcie_$i.txt")"
  grep -o "copy_engine=0x[0-9a-f]*" "$O/pcie_$i.log" | sort | uniq -c | head -8
  grep -o "free_engine_mask 0x[0-9a-f]*, rec_engine_mask 0x[0-9a-f]*" "$O/pcie_$i.log" | sort | uniq -c | head -8
  gzip -f "$O/pcie_$i.log"
done
