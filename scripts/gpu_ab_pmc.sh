#!/bin/bash
# A/B of library variants (syzkaller_amd/exp/lib*.so via SG_LIB_PATH): the
# bench's kernel times and the PMC traffic (FETCH_SIZE / WRITE_SIZE passes)
# of each, summarised per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-A B}; do
  export SG_LIB_PATH=$PWD/syzkaller_amd/exp/lib$v.so
  timeout -k 10 300 python -u bench.py --no-steady --no-cpu --no-from-traces > gpurun_out/abp_bench_$v.log 2>&1
  rc=$?; echo "$v bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/abp_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), {k: round(v['avg_ms'],3) for k, v in d['kernels'].items()})"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $C -d gpurun_out/abp_${C}_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-account --no-steady --no-from-traces > gpurun_out/abp_${C}_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $C rc=$rc"; exit $rc; }
  done
  python3 scripts/pmc_summary.py gpurun_out/abp_FETCH_SIZE_$v/run_counter_collection.csv gpurun_out/abp_WRITE_SIZE_$v/run_counter_collection.csv gpurun_out/abp_pmc_$v.json $v 2 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print({k: (round(x['fetch_bytes_x2']/1e9,2), round(x['write_bytes']/1e9,2)) for k,x in d['kernels'].items()})"
done
