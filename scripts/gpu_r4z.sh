#!/bin/bash
# r04: 64-edge windows as the default executor-exact kernel: its parity tests,
# the A0 row, and the bench's from-traces / steady legs (executor-exact lists).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4z}
timeout -k 10 600 python -u -m pytest tests/test_traces.py tests/test_gpu_parity.py tests/test_ipc.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_rows.py a0 > gpurun_out/${T}_a0.jsonl 2> gpurun_out/${T}_a0.err || exit 1
tail -1 gpurun_out/${T}_a0.jsonl | cut -c1-300
timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --no-cpu --no-host-api --no-account > gpurun_out/${T}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ft=d['from_traces']; st=d['steady_state']
print('c2', round(d['ms_per_step'],3), 'ft', round(ft['ms_per_step'],3), 'exec_exact', ft['executor_exact'])
print('steady traces', st.get('from_traces'))"
