#!/bin/bash
# The field-lane test, then the corpus P roundtrip at several long-slice split sizes (AVR_SPLIT_BYTES):
# MB/s, compress / decompress seconds and container bytes.  Each GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/split_sweep
mkdir -p $O
echo "== lane test" && timeout -k 10 400 python -u -m pytest tests/test_gpu_fields.py -k field_lane -x -q --timeout 300 \
  --timeout-method thread > $O/lane_test.log 2>&1 && tail -2 $O/lane_test.log || exit 1
for b in 131072 98304 81920 65536; do
  AVR_SPLIT_BYTES=$b REPS=3 timeout -k 10 200 python -u scripts/field_lane_ab.py > $O/s$b.json 2> $O/s$b.err \
    || { echo "split $b failed"; tail -5 $O/s$b.err; exit 1; }
  python3 -c "import json,statistics as st; d=json.load(open('$O/s$b.json')); print($b, round(d['MB_s'], 3), round(st.median(d['compress_s']), 3), round(st.median(d['decompress_s']), 3), d['avrc_bytes'], round(d['avrc_bytes'] / d['bytes'], 5))"
done
