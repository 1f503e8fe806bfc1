#!/bin/bash
# Iteration: gpu tests, the default bench (C2 only), a spill/geometry diagnostic
# of one partitioned step (SG_DEBUG_PART), the A0 row.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-iter2}
timeout -k 10 900 python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -x -v -p no:cacheprovider --timeout 600 \
  --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-steady ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
SG_DEBUG_PART=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-account --no-steady \
  > gpurun_out/dbg_$TAG.log 2>&1
rc=$?; echo "dbg rc=$rc"; grep "sg part" gpurun_out/dbg_$TAG.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_rows.py a0 > gpurun_out/rows_$TAG.log 2>&1
rc=$?; echo "rows rc=$rc"; tail -1 gpurun_out/rows_$TAG.log
exit $rc
