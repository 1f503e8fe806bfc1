#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r4l.sh && bash scripts/gpu_r4k.sh
