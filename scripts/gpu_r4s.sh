#!/bin/bash
# r04: the persistent prefetching pass-1 scatter (SG_P1_PF), parity then A/B on the C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4s}
SG_P1_PF=1 timeout -k 10 600 python -u -m pytest tests/test_c2_full.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest pf rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host-api --no-steady --no-from-traces --no-account"
for i in 1 2; do
  for pf in 0 1; do
    SG_P1_PF=$pf timeout -k 10 300 $B > gpurun_out/${T}_pf${pf}_$i.log 2>&1 || exit 1
    tail -1 gpurun_out/${T}_pf${pf}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pf=$pf', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items() if k in ('p1_scatter','p2_scatter','bucket_triage','p1_hist','p2_hist')})"
  done
done
