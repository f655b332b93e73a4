#!/bin/bash
# A/B timing of avrecode_amd/var/prev (last commit's build) against the working build, then the
# -m gpu suite on the working build:  gpurun -- 'bash scripts/gpu_ab_check.sh tag'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab}
timeout -k 10 500 python scripts/ab_time.py avrecode_amd/var/prev/libavrecode.so avrecode_amd/libavrecode.so > gpurun_out/${tag}_ab.log 2>&1
rc=$?
grep -v "^ \|^{\|^}" gpurun_out/${tag}_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log
exit $rc
