#!/bin/bash
# A/B timing of experiment builds (avrecode_amd/var/<name>/libavrecode.so) against the working
# build: gpurun -- 'bash scripts/gpu_ab_r04.sh tag name1 name2 ...'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
libs="avrecode_amd/libavrecode.so"
for v in "$@"; do libs="$libs avrecode_amd/var/$v/libavrecode.so"; done
timeout -k 10 1100 python scripts/ab_time.py $libs > gpurun_out/${tag}_ab.log 2>&1
rc=$?
grep -v "^ \|^{\|^}" gpurun_out/${tag}_ab.log
exit $rc
