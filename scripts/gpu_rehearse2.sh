#!/bin/bash
# Two-rank rehearsal of bench.py's C3 path on one GPU (gloo: RCCL refuses two
# ranks on one device; the driver's multi-GPU runs use RCCL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SG_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --programs 32768 \
  > gpurun_out/rehearse2.log 2>&1
rc=$?; echo "rehearse2 rc=$rc"; tail -1 gpurun_out/rehearse2.log | cut -c1-400
exit $rc
