#!/bin/bash
# r04: queued-lists exec signal + full-size row parity tests, then the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4h}
timeout -k 10 900 python -u -m pytest tests/test_traces.py tests/test_full_rows.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread --durations=0 > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|s call" gpurun_out/${T}_pytest.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${T}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d['steady_state'].get('from_traces')), json.dumps(d['host_api']))"
exit $rc
