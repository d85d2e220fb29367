#!/bin/bash
# Host-link pair rate against the NUMA placement of the process and its
# pinned pages: tools/ubench_pcie in 8 fresh processes, each printing the CPU
# it runs on and the node of its pinned pages, with the "H2D + D2H on two
# streams" rate; plus the GPU's NUMA node from sysfs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-numa_pcie}"
mkdir -p "$O"
cd "$R"
for f in /sys/class/drm/card*/device/numa_node; do echo "$f: $(cat $f 2>/dev/null)"; done 2>/dev/null | head -4
lscpu 2>/dev/null | grep -i "numa" | head -4
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 ./tools/ubench_pcie 64 > "$O/p_$i.txt" 2>&1 || { echo "UBENCH FAILED"; tail "$O/p_$i.txt"; exit 1; }
  echo "$i: $(grep '^cpu ' "$O/p_$i.txt") | $(grep 'H2D + D2H on two streams' "$O/p_$i.txt" | cut -c35-80)"
done
