#!/bin/bash
# A/B of library variants (syzkaller_amd/exp/lib*.so, scripts/build_variant.sh)
# on the steady-state step with the M0 filter forced (scripts/exp/steady_step.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-A}; do
  lib=$PWD/syzkaller_amd/exp/lib$v.so
  [ "$v" = "A" ] && lib=$PWD/syzkaller_amd/libsyzsig.so
  SG_LIB_PATH=$lib timeout -k 10 300 python -u scripts/exp/steady_step.py ${MODE:-1} 3 > gpurun_out/ab_steady_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -E "kernels|step" gpurun_out/ab_steady_$v.log | tail -2
  [ $rc -eq 0 ] || exit $rc
done
