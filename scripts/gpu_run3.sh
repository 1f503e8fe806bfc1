#!/bin/bash
# GPU pass: parity tests, smoke, bench (partitioned + diff path), kernel stats,
# PMC passes of a short bench and of the calibration kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01b}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --diff --no-cpu > gpurun_out/bench_diff.log 2>&1
rc=$?; echo "bench diff rc=$rc"; tail -1 gpurun_out/bench_diff.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"
[ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/pmc_${C}_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-account > gpurun_out/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmccal_${C}_$TAG -o run --output-format csv -- python3 scripts/pmc_calib.py > gpurun_out/pmccal_$C.log 2>&1
  rc=$?; echo "pmc calib $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
