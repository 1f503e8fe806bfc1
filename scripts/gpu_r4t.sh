#!/bin/bash
# r04: record-slice cuts on the device, no wait between slices: parity (slicing
# tests, C3 slice, shard, host pipeline), then C3 per-rank steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4t}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_traces.py tests/test_c3_slice.py tests/test_shard_gpu.py tests/test_host_pipeline.py tests/test_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --mode c3 --no-cpu --steps 6 --warmup 2"
for v in "fresh_plain:" "fresh_auto:--c3-two-phase" "steady_plain:--c3-steady" "steady_auto:--c3-steady --c3-two-phase"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 $B $a > gpurun_out/${T}_c3_$n.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$n', round(d['ms_per_step'],3), 'kernel sum', round(sum(v['ms_per_step'] for v in k.values()),3))"
done
