#!/bin/bash
# Builds syzkaller_amd/exp/lib$1.so: the library with sg_bucket.hip compiled
# under extra defines ($2, e.g. "-DSG_P2_ORDER=0"), for scripts/gpu_ab.sh.
set -e
cd "$(dirname "$0")/../syzkaller_amd"
make -s ARCH=gfx950 >/dev/null
mkdir -p ../build_exp exp
/opt/rocm/bin/hipcc -c -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-value -Wno-unused-result $2 \
  -o ../build_exp/sg_bucket_$1.o csrc/sg_bucket.hip
objs=$(ls build/*.o | grep -v sg_bucket.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o exp/lib$1.so $objs ../build_exp/sg_bucket_$1.o
