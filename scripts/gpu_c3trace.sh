#!/bin/bash
# C3 two-phase step at one rank under a kernel trace (both prefix forms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c3t}
for K in 0 1; do
SG_PREFIX_PAIRS=$K timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3trace_${T}_$K -o run -- python3 -u bench.py --mode c3 --c3-two-phase --steps 2 --warmup 1 > gpurun_out/c3trace_${T}_$K.log 2>&1
rc=$?; echo "pairs=$K rc=$rc"; tail -1 gpurun_out/c3trace_${T}_$K.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
SG_PREFIX_PAIRS=1 SG_DEBUG_PART=1 timeout -k 10 300 python3 -u bench.py --mode c3 --c3-two-phase --steps 1 --warmup 0 2>&1 | grep "sg prefix" > gpurun_out/c3pairs_$T.log
echo "pairs: $(head -2 gpurun_out/c3pairs_$T.log)"
