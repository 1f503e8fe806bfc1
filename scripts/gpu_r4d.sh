#!/bin/bash
# r04: pipelined map probing.  Parity of the bucket paths, then C2 bench and
# phase counters: register kernel with 2 / 1 pending probes, ring kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4d}
SG_BUCKET_RING=0 timeout -k 10 600 python -u -m pytest tests/test_c2_full.py tests/test_gpu_parity.py tests/test_traces.py tests/test_shard_gpu.py tests/test_c3_slice.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest reg rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_c2_full.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_ring.log 2>&1
rc=$?; echo "pytest ring rc=$rc"; tail -2 gpurun_out/${T}_pytest_ring.log
[ $rc -eq 0 ] || exit $rc
B="python -u bench.py --no-cpu --no-steady --no-from-traces"
for v in "reg2:SG_BUCKET_RING=0" "reg1:SG_BUCKET_RING=0 SG_LIB_PATH=syzkaller_amd/exp/libP1.so" "ring2:SG_BUCKET_RING=1"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 300 $B > gpurun_out/${T}_bench_$n.log 2>&1 || exit 1
  echo "$n $(tail -1 gpurun_out/${T}_bench_$n.log | grep -o '"ms_per_step": [0-9.]*')"
  env $e SG_DEBUG_PART=1 timeout -k 10 300 $B --steps 1 --warmup 1 --no-account > gpurun_out/${T}_dbg_$n.log 2>&1 || exit 1
  grep "sg bucket per" gpurun_out/${T}_dbg_$n.log | tail -1 | cut -c1-260
done
