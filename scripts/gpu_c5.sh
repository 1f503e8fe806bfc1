#!/bin/bash
# C5: the report tests and the c5 row (plain and staged scatter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k cover_uncovered -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_c5_$T.log 2>&1
rc=$?; echo "pytest c5 rc=$rc"; tail -2 gpurun_out/pytest_c5_$T.log; [ $rc -eq 0 ] || exit $rc
SG_REPORT_STAGED=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k cover_uncovered -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_c5s_$T.log 2>&1
rc=$?; echo "pytest c5 staged rc=$rc"; tail -2 gpurun_out/pytest_c5s_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_rows.py c5 > gpurun_out/rows_c5_$T.jsonl 2>&1
rc=$?; echo "rows c5 rc=$rc"; grep row gpurun_out/rows_c5_$T.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"kernels_ms\"], d[\"frac_hbm_query\"], d[\"parity_2M_prefix\"], d[\"pc_order\"])"; [ $rc -eq 0 ] || exit $rc
exit $rc
