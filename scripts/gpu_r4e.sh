#!/bin/bash
# r04: full GPU tests, the default bench, the C3 per-rank PMC section (two-phase
# prefix step at one rank), then the N=2 rehearsal through bench.py's own launcher.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${T}_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${c}_${T}c3 -o run --output-format csv -- python3 bench.py --mode c3 --c3-two-phase --steps 2 --warmup 1 --no-cpu --no-account > gpurun_out/pmc_${c}_${T}c3.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_${T}.json
python3 scripts/pmc_summary.py $(ls gpurun_out/pmc_FETCH_SIZE_${T}c3/run_counter_collection.csv) $(ls gpurun_out/pmc_WRITE_SIZE_${T}c3/run_counter_collection.csv) gpurun_out/pmc_traffic_${T}.json ${T}c3 c3 merge > gpurun_out/${T}_pmcsum.log 2>&1 || exit 1
cp gpurun_out/pmc_traffic_${T}.json profiles/pmc_traffic.json
SG_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --programs 16384 > gpurun_out/${T}_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/${T}_gloo2.log | cut -c1-300
exit $rc
