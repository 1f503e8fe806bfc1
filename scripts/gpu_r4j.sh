#!/bin/bash
# r04: global-atomic rates -- the random-address peak (micro), the claim path's
# kernel times, and its TCC_ATOMIC counts (separate PMC pass), summarised.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4j}
hipcc -O3 --offload-arch=gfx950 -o /tmp/atomics scripts/micro/atomics.hip 2>/dev/null || exit 1
timeout -k 10 300 /tmp/atomics > gpurun_out/${T}_atomics_micro.txt 2>&1 || exit 1
cat gpurun_out/${T}_atomics_micro.txt
timeout -k 10 400 python3 scripts/atomic_rate.py run gpurun_out/${T}_times.json > gpurun_out/${T}_run.log 2>&1
rc=$?; echo "run rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 -s KILL 400 rocprofv3 --pmc TCC_ATOMIC TCP_TOTAL_ATOMIC_WITH_RET TCP_TOTAL_ATOMIC_WITHOUT_RET -d gpurun_out/${T}_pmc -o run --output-format csv -- python3 scripts/atomic_rate.py run /tmp/at_pmc.json > gpurun_out/${T}_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/atomic_rate.py summary gpurun_out/${T}_times.json $(ls gpurun_out/${T}_pmc/run_counter_collection.csv) gpurun_out/${T}_atomics_micro.txt gpurun_out/${T}_atomics.json > /dev/null
python3 -c "import json; d=json.load(open('gpurun_out/${T}_atomics.json')); print(json.dumps({k:{kk:v[kk] for kk in ('avg_ms_events','atomics_per_s_G','frac_of_random_peak')} for k,v in d['kernels'].items()}))"
