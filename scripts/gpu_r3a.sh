#!/bin/bash
# Round-3 iteration: report-path tests, the C5 row, the two-stream overlap
# experiment (plain and with the bucket grid capped), then the GPU suite and
# the default bench.  Each step under its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r3a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k cover_uncovered -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_c5_$T.log 2>&1
rc=$?; echo "pytest c5 rc=$rc"; tail -2 gpurun_out/pytest_c5_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_rows.py c5 > gpurun_out/rows_c5_$T.jsonl 2>&1
rc=$?; echo "rows c5 rc=$rc"; cut -c1-700 gpurun_out/rows_c5_$T.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp/overlap.py > gpurun_out/overlap_$T.log 2>&1
rc=$?; echo "overlap rc=$rc"; cat gpurun_out/overlap_$T.log | tail -4; [ $rc -eq 0 ] || exit $rc
SG_BUCKET_BLOCKS=512 timeout -k 10 300 python -u scripts/exp/overlap.py > gpurun_out/overlap512_$T.log 2>&1
rc=$?; echo "overlap512 rc=$rc"; cat gpurun_out/overlap512_$T.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$T.log | cut -c1-400
exit $rc
