#!/bin/bash
# The slice batch's tail: walker lifetimes per slice against the launch span (AVR_PROFILE build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04l}
AVR_LIBRARY=avrecode_amd/prof/libavrecode.so timeout -k 10 300 python scripts/placement.py --slices 1024 --save gpurun_out/${tag}_place > gpurun_out/${tag}_placement.json 2> gpurun_out/${tag}_placement.err
rc=$?
cat gpurun_out/${tag}_placement.json; tail -3 gpurun_out/${tag}_placement.err
exit $rc
