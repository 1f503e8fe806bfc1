#!/bin/bash
# r04: per-bucket novelty counts (the single-counter atomics made the mark
# pass 3.3 ms), the two-barrier emitting flush, quad prefix-OR / set-OR
# passes: parity (shard/C3/pipeline tests), then C3 per-rank steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4n}
timeout -k 10 900 python -u -m pytest tests/test_bitmap_ops.py tests/test_shard_gpu.py tests/test_c3_slice.py tests/test_pipeline.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
B="python -u bench.py --mode c3 --no-cpu --steps 6 --warmup 2"
for v in "fresh_plain:" "fresh_auto:--c3-two-phase" "steady_plain:--c3-steady" "steady_auto:--c3-steady --c3-two-phase" "steady_kept:--c3-steady --c3-two-phase --c3-form kept" "fresh_kept:--c3-two-phase --c3-form kept"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 $B $a > gpurun_out/${T}_c3_$n.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],3), d.get('prefix_forms'), {a:round(b['ms_per_step'],3) for a,b in d['kernels'].items()})"
done
