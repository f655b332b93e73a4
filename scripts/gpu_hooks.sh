#!/bin/bash
# The hooks-surface GPU tests (tests/test_hooks.py) on the working build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-hooks}
timeout -k 10 600 python -u -m pytest tests/test_hooks.py -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -45
exit $rc
