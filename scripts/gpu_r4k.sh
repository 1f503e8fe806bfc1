#!/bin/bash
# r04: the prefix protocol's per-batch form (parity, then C3 per-rank steps at
# one rank: plain, two-phase auto/kept on fresh and steady batches), then the
# atomic-rate measurements (scripts/gpu_r4j.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4k}
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py tests/test_c3_slice.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
B="python -u bench.py --mode c3 --no-cpu --steps 6 --warmup 2"
for v in "fresh_plain:" "fresh_auto:--c3-two-phase" "fresh_kept:--c3-two-phase --c3-form kept" "steady_plain:--c3-steady" "steady_auto:--c3-steady --c3-two-phase" "steady_kept:--c3-steady --c3-two-phase --c3-form kept"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 $B $a > gpurun_out/${T}_c3_$n.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],3), d.get('prefix_forms'), d['config']['queued_frac'])"
done
TAG=${T}a bash scripts/gpu_r4j.sh
