#!/bin/bash
# r04: the LDS-ring bucket kernel. Bucket-path parity tests first, then the C2
# bench with the ring kernel (default) and the register kernel (SG_BUCKET_RING=0),
# then the debug phase counters of one launch of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4b}
timeout -k 10 600 python -u -m pytest tests/test_c2_full.py tests/test_gpu_parity.py tests/test_traces.py tests/test_shard_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-from-traces > gpurun_out/${T}_bench_ring.log 2>&1
rc=$?; echo "bench ring rc=$rc"; tail -1 gpurun_out/${T}_bench_ring.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
SG_BUCKET_RING=0 timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-from-traces > gpurun_out/${T}_bench_reg.log 2>&1
rc=$?; echo "bench reg rc=$rc"; tail -1 gpurun_out/${T}_bench_reg.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
SG_DEBUG_PART=1 timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-from-traces --steps 1 --warmup 1 --no-account > gpurun_out/${T}_dbg_ring.log 2>&1
rc=$?; echo "dbg rc=$rc"; grep "sg bucket" gpurun_out/${T}_dbg_ring.log | tail -4
exit $rc
