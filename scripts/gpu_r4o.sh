#!/bin/bash
# r04: pipelined C2 loop with the bucket stage and the next partition on
# disjoint CU sets (scripts/exp/cumask.py), several splits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4o}
for s in none lo:128 even odd8 lo:160 lo:96; do
  n=$(echo $s | tr ':' '_')
  BUCKET_CUS=$s timeout -k 10 300 python -u scripts/exp/cumask.py > gpurun_out/${T}_$n.log 2>&1 || { echo "fail $s"; tail -5 gpurun_out/${T}_$n.log; exit 1; }
  grep "rep 2" gpurun_out/${T}_$n.log; tail -1 gpurun_out/${T}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernels'])"
done
