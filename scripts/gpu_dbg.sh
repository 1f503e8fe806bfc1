#!/bin/bash
# Diagnostics only: one C2 step with the partitioned path's phase counters
# (SG_DEBUG_PART), then (unless NOBENCH=1) the default bench without the
# steady-state leg.  Outputs under gpurun_out/ with TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-dbg}
SG_DEBUG_PART=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 0 --no-cpu --no-account --no-steady \
  ${DBG_ARGS:-} > gpurun_out/dbg_$TAG.log 2>&1
rc=$?; echo "dbg rc=$rc"; grep -A3 "n=880" gpurun_out/dbg_$TAG.log | grep "sg bucket per\|sg part" | tail -4
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py --no-steady --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
fi
exit $rc
