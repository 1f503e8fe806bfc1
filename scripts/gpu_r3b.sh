#!/bin/bash
# C5 tests and row, then the two-stream overlap experiment (plain, bucket grid capped).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r3b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k cover_uncovered -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_c5_$T.log 2>&1
rc=$?; echo "pytest c5 rc=$rc"; tail -2 gpurun_out/pytest_c5_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_rows.py c5 > gpurun_out/rows_c5_$T.jsonl 2>&1
rc=$?; echo "rows c5 rc=$rc"; grep row gpurun_out/rows_c5_$T.jsonl | cut -c180-560; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp/overlap.py > gpurun_out/overlap_$T.log 2>&1
rc=$?; echo "overlap rc=$rc"; tail -4 gpurun_out/overlap_$T.log; [ $rc -eq 0 ] || exit $rc
for B in 512 256; do
SG_BUCKET_BLOCKS=$B timeout -k 10 300 python -u scripts/exp/overlap.py > gpurun_out/overlap${B}_$T.log 2>&1
rc=$?; echo "overlap$B rc=$rc"; tail -4 gpurun_out/overlap${B}_$T.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
