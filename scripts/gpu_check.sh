#!/bin/bash
# One GPU session: smoke, GPU tests, a small bench (+ whole-file roundtrips).  Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& tail -2 gpurun_out/smoke.log \
&& echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 \
&& tail -3 gpurun_out/pytest_gpu.log \
&& echo "== bench (small)" && timeout -k 10 600 python bench.py ${BENCH_ARGS:---slices 96 --steps 1 --warmup 1 --cpu-seconds 5} > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err \
&& cat gpurun_out/bench_small.json
rc=$?
[ $rc -ne 0 ] && { tail -30 gpurun_out/*.log gpurun_out/*.err 2>/dev/null; }
exit $rc
