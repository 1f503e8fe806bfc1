#!/bin/bash
# C5 random-order regrouping: parity, then the row with and without precomputed chunks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_full_rows.py -k "cover or c5" -m gpu > gpurun_out/c5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/c5_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  SG_REPORT_QCHUNK=$v timeout -k 10 120 python bench_rows.py c5 > gpurun_out/c5_q$v.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/c5_q$v.log') if l.startswith('{')][-1]); print('$v', round(d['device_ms_query_kernel'],3), {k: round(x,3) for k,x in d['kernels_ms'].items()})"
done
