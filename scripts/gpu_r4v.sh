#!/bin/bash
# r04: partition tiles of 8K entries (512- or 1024-thread blocks) against 16K
# (SG_LIB_PATH variants from scripts/build_variant.sh): C2 parity, then A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4v}
for v in PT8K PT8KW; do
  SG_LIB_PATH=$PWD/syzkaller_amd/exp/lib$v.so timeout -k 10 600 python -u -m pytest tests/test_c2_full.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -1 gpurun_out/${T}_pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
B="python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host-api --no-steady --no-from-traces --no-account"
for i in 1 2; do
  for v in base PT8K PT8KW; do
    L=""; [ "$v" != base ] && L="$PWD/syzkaller_amd/exp/lib$v.so"
    SG_LIB_PATH=$L timeout -k 10 300 $B > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    tail -1 gpurun_out/${T}_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items() if k in ('p1_scatter','p2_scatter','bucket_triage','p1_hist','p2_hist','scan')})"
  done
done
