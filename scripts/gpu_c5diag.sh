#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SG_LIB_PATH=$PWD/syzkaller_amd/exp/libdiag.so timeout -k 10 300 python -u bench_rows.py c5 > gpurun_out/rows_c5diag.jsonl 2>&1
rc=$?; echo "rows c5 diag rc=$rc"; grep row gpurun_out/rows_c5diag.jsonl | cut -c180-560; exit $rc
