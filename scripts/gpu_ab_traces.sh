#!/bin/bash
# A/B of library variants on the from-traces leg: its per-kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-A B}; do
  SG_LIB_PATH=$PWD/syzkaller_amd/exp/lib$v.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-steady --no-cpu \
    --no-host-api --no-account > gpurun_out/abt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/abt_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['from_traces']; print(round(f['ms_per_step'],3), {k: round(v['avg_ms'],3) for k, v in f['kernels'].items()})"
done
