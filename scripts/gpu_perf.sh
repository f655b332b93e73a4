#!/bin/bash
# Perf check: GPU tests (optional), the 1024-slice bench, and R-mode cockatoo roundtrip timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  echo "== pytest" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/pytest_perf.log 2>&1 && tail -2 gpurun_out/pytest_perf.log || { tail -30 gpurun_out/pytest_perf.log; exit 1; }
fi
echo "== bench" && timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-files --no-corpus > gpurun_out/bench_perf.json 2> gpurun_out/bench_perf.err \
&& python3 -c "import json;b=json.load(open('gpurun_out/bench_perf.json'));c=b['config'];print('bench', round(b['value'],2), 'MB/s compress', round(c['compress_ms'],1), 'decompress', round(c['decompress_ms'],1))" \
&& for m in "" "-p"; do timeout -k 10 120 ./avrecode_amd/recode roundtrip $m tests/fixtures/cockatoo.mp4 2>/dev/null | grep "compress "; done
