#!/bin/bash
# Trace path: its parity tests, then the bench's from_traces leg (no steady state / CPU legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-tr}
timeout -k 10 400 python -u -m pytest tests/test_traces.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_tr_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_tr_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --no-steady --no-cpu --no-account > gpurun_out/bench_tr_$T.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_tr_$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d['value']/1e9, {k: round(v['avg_ms'],3) for k, v in d['kernels'].items()}); ft=d.get('from_traces') or {}; print({k: ft[k] for k in ft if k in ('ms_per_step','raw_pcs_per_s','value','kernels')})"
exit $rc
