#!/bin/bash
# C3 per-rank: the prefix / shard GPU tests, then the plain and two-phase
# per-rank step at one rank (bench.py --mode c3; the two-phase step also in
# its SG_PREFIX_PAIRS form).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c3}
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_c3_slice.py tests/test_prefix.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_c3_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_c3_$T.log; [ $rc -eq 0 ] || exit $rc
for M in "" "--c3-two-phase" "pairs"; do
if [ "$M" = pairs ]; then A="--c3-two-phase"; K=1; else A=$M; K=0; fi
SG_PREFIX_PAIRS=$K timeout -k 10 500 python -u bench.py --mode c3 $A --steps 4 --warmup 1 > gpurun_out/bench_c3${M}_$T.log 2>&1
rc=$?; echo "c3 $M rc=$rc"; tail -1 gpurun_out/bench_c3${M}_$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), {k: round(v['avg_ms'],3) for k, v in d['kernels'].items()})"; [ $rc -eq 0 ] || exit $rc
done
