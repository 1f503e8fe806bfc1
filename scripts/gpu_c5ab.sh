#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in base ${VARIANTS:-T32}; do
  L=""; [ "$V" != base ] && L="$PWD/syzkaller_amd/exp/lib$V.so"
  SG_LIB_PATH=$L timeout -k 10 300 python -u bench_rows.py c5 > gpurun_out/rows_c5_$V.jsonl 2>&1
  rc=$?; echo "$V rc=$rc"; grep row gpurun_out/rows_c5_$V.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernels_ms']['report_chunks'], d['pc_order']['kernels_ms']['report_chunks'], d['frac_hbm_query'], d['pc_order']['frac_hbm_query'], d['parity_2M_prefix'], d['pc_order']['same_result'])"
  [ $rc -eq 0 ] || exit $rc
done
