#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 4; do
SG_MINIMIZE_FILTER_RANKS=$R timeout -k 10 300 python -u bench_rows.py c4 > gpurun_out/c4_R$R.jsonl 2>&1
rc=$?; echo "R=$R rc=$rc"; grep row gpurun_out/c4_R$R.jsonl | cut -c90-330; [ $rc -eq 0 ] || exit $rc
done
