#!/bin/bash
# r04: non-temporal stores in the partition scatters (SG_NT_STORE), A/B on the C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4r}
B="python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host-api --no-steady --no-from-traces --no-account"
for i in 1 2; do
  for nt in 0 1; do
    SG_NT_STORE=$nt timeout -k 10 300 $B > gpurun_out/${T}_nt${nt}_$i.log 2>&1 || exit 1
    tail -1 gpurun_out/${T}_nt${nt}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nt=$nt', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items() if k in ('p1_scatter','p2_scatter','bucket_triage','p1_hist','p2_hist')})"
  done
done
SG_NT_STORE=1 timeout -k 10 600 python -u -m pytest tests/test_c2_full.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest nt rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; exit $rc
