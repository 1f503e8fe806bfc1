#!/bin/bash
# producer-wave slot-region executor kernel: parity (crafted + random + golden + queued lists), then a0 timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k exec_signal -m gpu > gpurun_out/ex2_tests.log 2>&1 || { tail -30 gpurun_out/ex2_tests.log; exit 1; }
tail -2 gpurun_out/ex2_tests.log
for r in ${ROWS:-104 102 0 104}; do
  SG_EXEC_REGION=$r timeout -k 10 120 python bench_rows.py a0 > gpurun_out/ex2_a0_$r.log 2>&1 || exit 1
  echo "$r $(grep -o '"exec_signal": [0-9.]*' gpurun_out/ex2_a0_$r.log | head -1)"
done
