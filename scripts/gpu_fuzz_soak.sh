#!/bin/bash
# fuzzer soak: RS16_FUZZ_MULT x the default cases at several seeds (each a fresh pytest process)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${1:-soak}"
mkdir -p "$O"
cd "$R"
for seed in ${SEEDS:-1 2 3}; do
  RS16_FUZZ_SEED=$seed RS16_FUZZ_MULT=${MULT:-8} timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > "$O/seed$seed.log" 2>&1 || { echo "SOAK FAILED seed $seed"; tail -30 "$O/seed$seed.log"; exit 1; }
  echo "seed $seed: $(tail -1 "$O/seed$seed.log")"
done
