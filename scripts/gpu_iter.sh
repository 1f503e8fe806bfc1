#!/bin/bash
# Quick GPU iteration: triage parity tests, then the default bench (no CPU
# baseline), then a kernel-trace profile of a short bench.  TAG names outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-iter}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${TESTS:-triage}" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-account > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/extra_$TAG.log 2>&1
  rc=$?; echo "extra rc=$rc"; tail -${EXTRA_TAIL:-8} gpurun_out/extra_$TAG.log | cut -c1-300
fi
exit $rc
