#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_trace.sh || exit $?
TAG=c3b bash scripts/gpu_c3.sh
