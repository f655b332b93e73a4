#!/bin/bash
# BASELINE configs[3] at its full size (600 s of 4K, ~4.5 GB) at N = 1: one warm-up + one timed
# step of bench.py --stream-shard, with a heartbeat file so a long parse is not taken for a hang.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04}
( while true; do date +%T >> gpurun_out/stream600_${tag}_hb.txt; sleep 30; done ) &
hb=$!
timeout -k 10 1080 python -u bench.py --stream-shard --stream-seconds 600 --steps 1 --warmup 1 \
  > gpurun_out/stream600_${tag}.json 2> gpurun_out/stream600_${tag}.err
rc=$?
kill $hb
tail -30 gpurun_out/stream600_${tag}.err
cat gpurun_out/stream600_${tag}.json
exit $rc
