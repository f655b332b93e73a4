#!/bin/bash
# Round 4: hooks / streaming / distributed-bench GPU tests, then A/B of the decoder variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== hooks + dist tests" && timeout -k 10 900 python -u -m pytest tests/test_hooks.py tests/test_gpu_bench_dist.py -m gpu -v --timeout 420 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?
tail -22 gpurun_out/r04c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
shift; echo "== A/B" && bash scripts/gpu_ab_r04.sh r04c "$@"
