#!/bin/bash
# A/B of library variants (syzkaller_amd/exp/lib*.so via SG_LIB_PATH): the
# phase diagnostics and the bench (no steady state, no CPU leg) for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-A B}; do
  SG_LIB_PATH=$PWD/syzkaller_amd/exp/lib$v.so SG_DEBUG_PART=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 0 \
    --no-cpu --no-account --no-steady > gpurun_out/ab_dbg_$v.log 2>&1
  rc=$?; echo "$v dbg rc=$rc"; grep "sg bucket per" gpurun_out/ab_dbg_$v.log | tail -1
  [ $rc -eq 0 ] || exit $rc
  SG_LIB_PATH=$PWD/syzkaller_amd/exp/lib$v.so timeout -k 10 300 python -u bench.py --no-steady --no-cpu ${BENCH_ARGS:-} \
    > gpurun_out/ab_bench_$v.log 2>&1
  rc=$?; echo "$v bench rc=$rc"
  tail -1 gpurun_out/ab_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), {k: round(v['avg_ms'],3) for k, v in d['kernels'].items()})"
  [ $rc -eq 0 ] || exit $rc
done
