#!/bin/bash
# r04: host -> device staging rates (scripts/micro/h2d.hip), 1 GiB and 3.5 GB
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
hipcc -O3 --offload-arch=gfx950 -o /tmp/h2d scripts/micro/h2d.hip 2>/dev/null || exit 1
timeout -k 10 300 /tmp/h2d 1073741824 > gpurun_out/r4f_h2d.txt 2>&1 || exit 1
timeout -k 10 300 /tmp/h2d 3500000000 >> gpurun_out/r4f_h2d.txt 2>&1
rc=$?; cat gpurun_out/r4f_h2d.txt; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; exit $rc
