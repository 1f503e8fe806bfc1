#!/bin/bash
# r04: the lean pass-1 histogram -- parity (full C2 tests with SG_HIST_LEAN=1),
# then two C2 triages on two streams (scripts/exp/overlap.py) with the default
# and the lean histogram.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4l}
SG_HIST_LEAN=1 timeout -k 10 600 python -u -m pytest tests/test_c2_full.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest lean rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
NB=8 timeout -k 10 300 python -u scripts/exp/overlap.py > gpurun_out/${T}_overlap.log 2>&1 || exit 1
cat gpurun_out/${T}_overlap.log | grep rep
SG_HIST_LEAN=1 NB=8 timeout -k 10 300 python -u scripts/exp/overlap.py > gpurun_out/${T}_overlap_lean.log 2>&1 || exit 1
cat gpurun_out/${T}_overlap_lean.log | grep rep
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${T}_pipe_pytest.log 2>&1
rc=$?; echo "pytest pipeline rc=$rc"; tail -2 gpurun_out/${T}_pipe_pytest.log
[ $rc -eq 0 ] || exit $rc
B="python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host-api --no-steady --no-from-traces --no-account --pipeline"
timeout -k 10 400 $B > gpurun_out/${T}_bench_pipe.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_pipe.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seq', d['ms_per_step'], 'pipe', d['pipelined'])"
SG_HIST_LEAN=1 timeout -k 10 400 $B > gpurun_out/${T}_bench_pipe_lean.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_pipe_lean.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lean seq', d['ms_per_step'], 'pipe', d['pipelined'])"
