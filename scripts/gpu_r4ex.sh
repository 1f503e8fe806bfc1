#!/bin/bash
# slot-region executor kernel: parity, then the a0 row per window size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k exec_signal tests/test_traces.py -m gpu > gpurun_out/ex_tests.log 2>&1 || exit 1
for r in 0 1 2 4 8 16; do
  SG_EXEC_REGION=$r timeout -k 10 120 python bench_rows.py a0 > gpurun_out/ex_a0_$r.log 2>&1 || exit 1
done
