#!/bin/bash
# r04 first call: validate the u32-scan RPC decode (test_rpc + the f4 row) and
# run the extended MALL/L2 reuse microbenchmark.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rpc.py -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/r4a_rpc.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r4a_rpc.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench_rows.py f4 > gpurun_out/r4a_rows.log 2>&1
rc=$?; echo "rows rc=$rc"; tail -2 gpurun_out/r4a_rows.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
hipcc -O3 --offload-arch=gfx950 -o /tmp/mall_reuse scripts/micro/mall_reuse.hip 2>/dev/null || exit 1
timeout -k 10 300 /tmp/mall_reuse > gpurun_out/r4a_mall.txt 2>&1
rc=$?; echo "mall rc=$rc"; cat gpurun_out/r4a_mall.txt
exit $rc
