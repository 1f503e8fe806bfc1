#!/bin/bash
# Round profile: all GPU tests, smoke, the default bench, the same default
# bench under rocprofv3 --kernel-trace --stats, and separate FETCH_SIZE /
# WRITE_SIZE PMC passes over a short bench (plus the calibration kernels).
# Outputs under gpurun_out/, TAG names them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
[ -n "$NOTEST" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOPROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_bench_$TAG.log 2>&1
  rc=$?; echo "rocprof stats rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOROWS" ]; then
  timeout -k 10 900 python -u bench_rows.py > gpurun_out/rows_$TAG.jsonl 2> gpurun_out/rows_$TAG.err
  rc=$?; echo "rows rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
[ -n "$NOPMC" ] && exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_${C}_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-account > gpurun_out/pmc_${C}_$TAG.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
