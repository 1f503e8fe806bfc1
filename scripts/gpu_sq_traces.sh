#!/bin/bash
# SQ counters over the from-traces leg's kernels (one pass of 8 SQ counters)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS \
  -d gpurun_out/sq_tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-steady --no-cpu --no-host-api --no-account > gpurun_out/sq_tr.log 2>&1
rc=$?; echo "sq rc=$rc"; exit $rc
