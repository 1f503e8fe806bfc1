#!/bin/bash
# One GPU iteration, each step under its own time limit, stopping at the first
# failure: pytest ($PYTEST_ARGS, default all -m gpu tests; NOTEST=1 skips), the
# bench ($BENCH_ARGS; NOBENCH=1 skips), an optional second bench ($BENCH2 =
# bench.py args), optional bench_rows.py rows ($ROWS = its args, e.g. "c5 f4"),
# and an optional rocprofv3 kernel trace of a short bench (PROF=1).  TAG names
# the outputs under gpurun_out/.  The parameterised runner for every
# iteration (the round profile is gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-iter}
if [ -z "$NOTEST" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH2" ]; then
  timeout -k 10 600 python -u bench.py $BENCH2 > gpurun_out/bench2_$TAG.log 2>&1
  rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2_$TAG.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$ROWS" ]; then
  timeout -k 10 900 python -u bench_rows.py $ROWS > gpurun_out/rows_$TAG.jsonl 2> gpurun_out/rows_$TAG.err
  rc=$?; echo "rows rc=$rc"; grep -c row gpurun_out/rows_$TAG.jsonl
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu --no-account --no-steady > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
