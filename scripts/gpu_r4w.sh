#!/bin/bash
# r04: the executor-exact kernel with K positions per lane (SG_EXEC_K = 2, 3,
# 4: windows of 64 K edges): parity, then the A0 row and the steady queued
# lists per K.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4w}
for k in 32 48; do
  SG_EXEC_K=$k timeout -k 10 600 python -u -m pytest tests/test_traces.py tests/test_gpu_parity.py -k "exec or traces" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_$k.log 2>&1
  rc=$?; echo "pytest K=$k rc=$rc"; tail -1 gpurun_out/${T}_pytest_$k.log; [ $rc -eq 0 ] || exit $rc
done
for k in 1 32 48; do
  SG_EXEC_K=$k timeout -k 10 300 python -u bench_rows.py a0 > gpurun_out/${T}_a0_$k.jsonl 2> gpurun_out/${T}_a0_$k.err || exit 1
  tail -1 gpurun_out/${T}_a0_$k.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=$k', d['kernels_ms'], round(d['pcs_per_s']/1e9,1))"
done
