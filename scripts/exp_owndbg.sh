cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in ${VARS:-0 15 31 16}; do
  SG_OWN_DBG=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-steady --no-from-traces --no-host-api > gpurun_out/owndbg_$v.log 2>&1 || exit 1
  echo "v=$v $(tail -1 gpurun_out/owndbg_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d['ordered_outputs']; print(round(o['kernels']['owned_sweep']['ms_per_step'],3))")"
done
