#!/bin/bash
# The round profile: all GPU tests, smoke, the default bench, the same bench
# under rocprofv3 --kernel-trace --stats, bench_rows.py, the FETCH_SIZE /
# WRITE_SIZE PMC passes of the C2 bench (sections c2, from_traces, steady) and
# of the C3 two-phase per-rank step (section c3), their summary into
# profiles/pmc_traffic.json of this copy, the default bench again (reading
# it), and the N=2 gloo rehearsal through bench.py's own launcher.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$T.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_bench_$T.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -z "$NOROWS" ]; then
  timeout -k 10 900 python -u bench_rows.py > gpurun_out/rows_$T.jsonl 2> gpurun_out/rows_$T.err
  rc=$?; echo "rows rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_${C}_$T -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-account > gpurun_out/pmc_${C}_$T.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C -d gpurun_out/pmc_${C}_${T}c3 -o run --output-format csv -- python3 bench.py --mode c3 --c3-two-phase --steps 2 --warmup 1 --no-cpu --no-account > gpurun_out/pmc_${C}_${T}c3.log 2>&1
  rc=$?; echo "pmc c3 $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
F=$(find gpurun_out/pmc_FETCH_SIZE_$T -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/pmc_WRITE_SIZE_$T -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py "$F" "$W" gpurun_out/pmc_traffic.json $T > gpurun_out/pmcsum_$T.log 2>&1 || exit 1
F=$(find gpurun_out/pmc_FETCH_SIZE_${T}c3 -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/pmc_WRITE_SIZE_${T}c3 -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py "$F" "$W" gpurun_out/pmc_traffic.json ${T}c3 c3 merge >> gpurun_out/pmcsum_$T.log 2>&1 || exit 1
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
echo "pmc summary done"
timeout -k 10 600 python -u bench.py --pipeline > gpurun_out/bench_$T.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$T.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --mode c3 --c3-two-phase > gpurun_out/bench_c3_$T.log 2>&1
rc=$?; echo "bench c3 rc=$rc"; tail -1 gpurun_out/bench_c3_$T.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
SG_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --programs 16384 > gpurun_out/gloo2_$T.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/gloo2_$T.log | cut -c1-300
exit $rc
