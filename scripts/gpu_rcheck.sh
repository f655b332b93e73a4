#!/bin/bash
# GPU check used while tuning the walker: the whole -m gpu suite, then the reference-model
# decompress section profile of cockatoo (needs `make -C avrecode_amd prof` beforehand).
#   gpurun -- 'bash scripts/gpu_rcheck.sh [tag]'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-rcheck}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
AVR_LIBRARY=avrecode_amd/prof/libavrecode.so timeout -k 10 200 python scripts/prof_rmode.py > gpurun_out/${tag}_prof_rmode.json 2>&1 \
  && cat gpurun_out/${tag}_prof_rmode.json
