#!/bin/bash
# Round 4: the hooks / streaming / bench-distributed GPU tests, then the section profile of the
# u64-coder decompress (AVR_PROFILE build) on the headline batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== hooks + dist tests" && timeout -k 10 900 python -u -m pytest tests/test_hooks.py tests/test_gpu_bench_dist.py -m gpu -v --timeout 420 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04b_tests.log
[ $rc -eq 0 ] || exit $rc
echo "== section profile (u64 coder)" && AVR_LIBRARY=avrecode_amd/prof/libavrecode.so timeout -k 10 300 python scripts/prof_sections.py --slices 1024 > gpurun_out/r04b_sections.json 2> gpurun_out/r04b_sections.err
rc=$?
cat gpurun_out/r04b_sections.json | head -60
exit $rc
