cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in base e2 e3; do
if [ $v = base ]; then unset SG_LIB_PATH; else export SG_LIB_PATH=$PWD/build_exp/lib_$v.so; fi
timeout -k 10 300 python bench.py --no-cpu --no-account > gpurun_out/b_$v.log 2>&1 || { tail -5 gpurun_out/b_$v.log; exit 1; }
python - <<PY
import json
d=json.loads(open('gpurun_out/b_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items() if 'avg_ms' in v})
PY
done
