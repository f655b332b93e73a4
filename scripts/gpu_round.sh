#!/bin/bash
# One GPU session: smoke, GPU parity tests, the default bench, and a rocprofv3 kernel-trace
# summary of the bench.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r04}
echo "== smoke" && timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& tail -2 gpurun_out/smoke.log \
&& echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& tail -3 gpurun_out/pytest_gpu.log \
&& echo "== bench" && timeout -k 10 900 python bench.py ${BENCH_ARGS:---cpu-seconds 10} > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& cat gpurun_out/bench.json \
&& echo "== rocprof" && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-files --no-corpus > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err \
&& cat gpurun_out/bench_prof.json
rc=$?
[ $rc -ne 0 ] && { tail -30 gpurun_out/*.log gpurun_out/*.err 2>/dev/null; }
exit $rc
