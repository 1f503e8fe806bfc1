#!/bin/bash
# r04: bucket-kernel phase counters (SG_DEBUG_PART) for the ring kernel (3 and
# 2 rounds in flight) and the register kernel, and the C2 bench of the 2-round ring.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4c}
B="python -u bench.py --no-cpu --no-steady --no-from-traces"
SG_DEBUG_PART=1 timeout -k 10 300 $B --steps 1 --warmup 1 --no-account > gpurun_out/${T}_dbg_r3.log 2>&1 || exit 1
grep "sg bucket" gpurun_out/${T}_dbg_r3.log | tail -2
SG_LIB_PATH=syzkaller_amd/exp/libR2.so SG_DEBUG_PART=1 timeout -k 10 300 $B --steps 1 --warmup 1 --no-account > gpurun_out/${T}_dbg_r2.log 2>&1 || exit 1
grep "sg bucket" gpurun_out/${T}_dbg_r2.log | tail -2
SG_BUCKET_RING=0 SG_DEBUG_PART=1 timeout -k 10 300 $B --steps 1 --warmup 1 --no-account > gpurun_out/${T}_dbg_reg.log 2>&1 || exit 1
grep "sg bucket" gpurun_out/${T}_dbg_reg.log | tail -2
SG_LIB_PATH=syzkaller_amd/exp/libR2.so timeout -k 10 300 $B > gpurun_out/${T}_bench_r2.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_bench_r2.log | cut -c1-200
