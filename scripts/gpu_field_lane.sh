#!/bin/bash
# The field lane on the GPU: the field / corpus / split tests, then the corpus P roundtrip with the lane
# off and on, twice each.  Each GPU step under its own time limit; the first failure ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/field_lane
mkdir -p $O
echo "== tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu_fields.py tests/test_gpu_files.py tests/test_gpu_split.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log || exit 1
for r in 1 2; do
  for v in 0 1; do
    AVR_FIELD_LANE=$v timeout -k 10 200 python -u scripts/field_lane_ab.py > $O/lane${v}_$r.json 2> $O/lane${v}_$r.err \
      || { echo "lane $v failed"; tail -5 $O/lane${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/lane${v}_$r.json')); print('lane', d['field_lane'], round(d['MB_s'], 3), [round(x, 3) for x in d['compress_s']], [round(x, 3) for x in d['decompress_s']], d['avrc_bytes'])"
  done
done
