#!/bin/bash
# Round 4 first GPU pass: the headline batch on the u64 coder (with the P32 extra), smoke, GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench (batch only)" && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files --no-corpus > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err \
&& cat gpurun_out/r04a_bench.json \
&& echo "== smoke" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 \
&& tail -1 gpurun_out/r04a_smoke.log \
&& echo "== pytest -m gpu" && timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > gpurun_out/r04a_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r04a_gpu_tests.log 2>/dev/null
exit $rc
