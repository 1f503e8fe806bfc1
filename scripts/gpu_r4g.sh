#!/bin/bash
# r04: the pipelined host ingest -- its parity tests, the host-path tests that
# already existed, then the bench's host_api leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4g}
timeout -k 10 900 python -u -m pytest tests/test_host_pipeline.py tests/test_gpu_parity.py tests/test_traces.py tests/test_cpp_mirror.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu --no-steady --no-from-traces --steps 4 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${T}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d['host_api']))"
exit $rc
