#!/bin/bash
# Report (C5) and Minimize (C4): their parity tests, then their rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-rows2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "minimize" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_rows2_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_rows2_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench_rows.py c4 > gpurun_out/rows2_$T.jsonl 2>&1
rc=$?; echo "rows rc=$rc"; grep row gpurun_out/rows2_$T.jsonl | cut -c1-900
exit $rc
