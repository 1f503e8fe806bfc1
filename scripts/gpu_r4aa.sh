#!/bin/bash
# r04: the executor-exact kernel comparing up to N writers of a pass directly
# (SG_EXEC_DIRECT; default build 8, variants 1 / 4 / 16): parity, A0 row.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4aa}
timeout -k 10 600 python -u -m pytest tests/test_traces.py tests/test_gpu_parity.py -k "exec or traces" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
SG_LIB_PATH=$PWD/syzkaller_amd/exp/libXD16.so timeout -k 10 600 python -u -m pytest tests/test_traces.py tests/test_gpu_parity.py -k "exec or traces" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest16.log 2>&1
rc=$?; echo "pytest XD16 rc=$rc"; tail -1 gpurun_out/${T}_pytest16.log; [ $rc -eq 0 ] || exit $rc
for v in base XD1 XD4 XD16; do
  L=""; [ "$v" != base ] && L="$PWD/syzkaller_amd/exp/lib$v.so"
  SG_LIB_PATH=$L timeout -k 10 300 python -u bench_rows.py a0 > gpurun_out/${T}_a0_$v.jsonl 2> gpurun_out/${T}_a0_$v.err || exit 1
  tail -1 gpurun_out/${T}_a0_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['kernels_ms'], round(d['pcs_per_s']/1e9,1))"
done
