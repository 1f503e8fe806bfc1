cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in ${VARS:-0 15}; do
  SG_OWN_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/owntr_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-steady --no-from-traces --no-host-api > gpurun_out/owntr_$v.log 2>&1 || exit 1
  echo "v=$v"; grep -E "k_own|k_rs_|k_bucket<false, true>|k_scatter|fillBuffer" gpurun_out/owntr_$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
done
