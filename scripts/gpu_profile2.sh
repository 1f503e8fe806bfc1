#!/bin/bash
# Round profile, second call: the bench under rocprofv3 --kernel-trace --stats,
# bench_rows.py, the FETCH_SIZE / WRITE_SIZE PMC passes, their summary
# (gpurun_out/pmc_traffic.json, also placed in profiles/ of this copy), then
# the default bench again so its roofline.traffic reads that summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03b}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench_rows.py > gpurun_out/rows_$TAG.jsonl 2> gpurun_out/rows_$TAG.err
rc=$?; echo "rows rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_${C}_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-account > gpurun_out/pmc_${C}_$TAG.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
F=$(find gpurun_out/pmc_FETCH_SIZE_$TAG -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/pmc_WRITE_SIZE_$TAG -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py "$F" "$W" gpurun_out/pmc_traffic.json $TAG > /dev/null && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
rc=$?; echo "pmc summary rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench2_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench2_$TAG.log | cut -c1-300
exit $rc
