#!/bin/bash
# rows A/B (base / x / y) with parity on x, then the stamps of the x build's column codec
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TESTS="tests/test_gpu_col.py tests/test_gpu_fuzz.py tests/test_gpu_rate.py tests/test_gpu_decode_check.py" VARIANTS="base x y" REPS=2 bash scripts/gpu_rows_ab.sh ${1:-r5an} || exit 1
bash scripts/gpu_r5ah.sh ${1:-r5an}_st | tail -1 | cut -c1-600
