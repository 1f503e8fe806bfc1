#!/bin/bash
# GPU pass: parity tests, smoke, default bench (+ optional extra commands in $EXTRA).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
if [ -n "$EXTRA" ]; then
  timeout -k 10 900 bash -c "$EXTRA" > gpurun_out/extra.log 2>&1
  rc=$?; echo "extra rc=$rc"; tail -5 gpurun_out/extra.log | cut -c1-400
fi
exit $rc
