#!/bin/bash
# PMC passes over an arbitrary python command ($CMD, e.g. "bench_rows.py a0"):
# one rocprofv3 run per counter group ($PASSES: groups ';', counters ',').
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pmccmd}
IFS=';' read -ra GROUPS_ <<< "$PASSES"
i=0
for g in "${GROUPS_[@]}"; do
  ctrs=${g//,/ }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 $CMD > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i ($g) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
exit 0
