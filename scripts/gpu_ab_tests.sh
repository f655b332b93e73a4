#!/bin/bash
# One GPU session for a kernel change: smoke, A/B timing of avrecode_amd/var/prev (the previous
# build) against the working build, then the -m gpu suite.  Every step has its own time limit and
# the chain stops at the first failure (no GPU step after a fault or a timeout).
#   gpurun -- 'bash scripts/gpu_ab_tests.sh tag'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-ab}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
&& tail -n 1 gpurun_out/${tag}_smoke.log \
&& timeout -k 10 400 python scripts/ab_time.py avrecode_amd/var/prev/libavrecode.so avrecode_amd/libavrecode.so > gpurun_out/${tag}_ab.log 2>&1 \
&& grep -v "^ \|^{\|^}" gpurun_out/${tag}_ab.log \
&& timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -n 12 gpurun_out/${tag}_*.log
exit $rc
