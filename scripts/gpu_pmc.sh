#!/bin/bash
# PMC passes over a short bench: one rocprofv3 run per counter group ($PASSES,
# groups separated by ';', counters in a group by ',').  TAG names outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pmc}
if [ -n "$LIST" ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
fi
IFS=';' read -ra GROUPS_ <<< "$PASSES"
i=0
for g in "${GROUPS_[@]}"; do
  ctrs=${g//,/ }
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-account ${BENCH_ARGS:-} > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i ($g) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
exit 0
