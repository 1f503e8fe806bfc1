#!/bin/bash
# rocprofv3 kernel trace + stats of one python command ($CMD); TAG names the output.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-prof}
timeout -k 10 ${LIMIT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 $CMD > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/prof_$T -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -d, -f1-6 "$f" | head -${TOP:-30}
exit $rc
