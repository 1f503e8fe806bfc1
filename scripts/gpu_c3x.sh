#!/bin/bash
# The C3 exchange forms rehearsed on one GPU: two ranks over gloo
# (SG_BENCH_BACKEND=gloo; RCCL needs a GPU per rank), a steady-state C3
# batch, the prefix protocol's exchange forced dense (bitmaps), sparse
# (candidate lists) and auto; each line's exchange_bytes_per_rank_per_step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c3x}
for X in ${FORMS:-dense sparse auto}; do
  SG_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --mode c3 --c3-steady --c3-exchange $X \
    --programs ${PROGRAMS:-16384} --steps 3 --warmup 1 --no-cpu > gpurun_out/c3x_${X}_$T.log 2>&1
  rc=$?; echo "c3 exchange $X rc=$rc"
  tail -1 gpurun_out/c3x_${X}_$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d['exchange_bytes_per_rank_per_step'], d['exchange_forms'])"
  [ $rc -eq 0 ] || exit $rc
done
