#!/bin/bash
# Host-batch copy diagnosis: tools/ubench_pcie (copy-engine
# and copy-kernel pairs, and H2D / D2H on every pair of 4 streams), then
# rocprofv3 kernel + memory-copy traces of scripts/probe_hb_cause.py in fresh
# processes (no preamble), so the copies of a slow and a fast process can be
# compared.  Every GPU step has its own time limit; the first failure ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-hbtrace}"
mkdir -p "$O"
cd "$R"
for i in 1 2; do
  timeout -k 10 120 ./tools/ubench_pcie 64 > "$O/pcie_$i.txt" 2>&1 || { echo "UBENCH FAILED"; tail "$O/pcie_$i.txt"; exit 1; }
done
cat "$O/pcie_1.txt"
for i in 1 2 3; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/tr_$i" \
      -o run --output-format csv -- python3 "$R/scripts/probe_hb_cause.py" none > "$O/tr_$i.log" 2>&1) \
      || { echo "TRACE FAILED"; tail -20 "$O/tr_$i.log"; exit 1; }
  grep "rep 3" "$O/tr_$i.log"
done
echo HBTRACE_DONE
