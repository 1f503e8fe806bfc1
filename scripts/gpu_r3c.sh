#!/bin/bash
# trace tests + from_traces bench, then the report tests and the c5 row
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_trace.sh || exit $?
TAG=c5f bash scripts/gpu_c5.sh
