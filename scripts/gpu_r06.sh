#!/bin/bash
# Round-6 GPU steps (each under its own time limit; the first failure ends the script):
#   golden   the oracle's answer for the bench headline batch -> gpurun_out/bench_batch.json
#            (copied to tests/golden/ for the tests of this call)
#   tests    the GPU tests named in TESTS (default: the round's new and changed ones)
#   bench    a short default bench run (BENCH_ARGS)
# STEPS selects (default "golden tests").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-"golden tests"}
TAG=${TAG:-r06}
for s in $STEPS; do
  case $s in
    golden)
      echo "== golden"
      timeout -k 10 600 python -u tests/golden/make_bench_golden.py gpurun_out/bench_batch.json \
        > gpurun_out/${TAG}_golden.log 2>&1 || { echo "golden failed rc=$?"; tail -20 gpurun_out/${TAG}_golden.log; exit 1; }
      cp gpurun_out/bench_batch.json tests/golden/bench_batch.json
      tail -3 gpurun_out/${TAG}_golden.log ;;
    tests)
      echo "== tests ${TESTS:-default}"
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        ${TESTS:-tests/test_gpu_chained.py tests/test_gpu_queue.py tests/test_gpu_parity.py} \
        > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
      tail -3 gpurun_out/${TAG}_tests.log ;;
    bench)
      echo "== bench ${BENCH_ARGS}"
      timeout -k 10 1000 python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
        || { echo "bench failed rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      tail -c 600 gpurun_out/${TAG}_bench.json ;;
  esac
done
echo "done"
