#!/bin/bash
# Builds syzkaller_amd/exp/lib$1.so: the library with one source file ($SRC,
# default sg_bucket) compiled under extra defines ($2, e.g. "-DSG_LDS_BARRIER=1"),
# for the A/B scripts (SG_LIB_PATH).
set -e
SRC=${SRC:-sg_bucket}
cd "$(dirname "$0")/../syzkaller_amd"
make -s ARCH=gfx950 >/dev/null
mkdir -p ../build_exp exp
/opt/rocm/bin/hipcc -c -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-value -Wno-unused-result $2 \
  -o ../build_exp/${SRC}_$1.o csrc/$SRC.hip
objs=$(ls build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o exp/lib$1.so $objs ../build_exp/${SRC}_$1.o
