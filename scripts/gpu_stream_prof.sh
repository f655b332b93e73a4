#!/bin/bash
# configs[3]'s kernels (the persistent queue kernel on the 600-s 4K stream) measured like the
# headline's: one timed stream step (bench.py --stream-shard, N = 1, phases), a rocprofv3 kernel
# trace with stats of the same command, and PMC passes (FETCH_SIZE, WRITE_SIZE, SQ mix), one counter
# group per run.  Output under gpurun_out/<TAG>_*; scripts/pmc_traffic.py --leg stream_shard turns
# the passes into profiles/<round>_stream_pmc.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_stream}
SECS=${SECS:-600}
ARGS="--stream-shard --stream-seconds $SECS --steps 1"
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_STEP" ]; then
  echo "== timed step (warm-up 1)"
  timeout -k 10 600 python3 -u bench.py $ARGS --warmup 1 > gpurun_out/$TAG/step.json 2> gpurun_out/$TAG/step.err \
    || { echo "step failed rc=$?"; tail -20 gpurun_out/$TAG/step.err; exit 1; }
  tail -c 1500 gpurun_out/$TAG/step.json
fi
echo "== kernel trace + stats"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- \
  python3 -u bench.py $ARGS --warmup 0 > gpurun_out/$TAG/trace.json 2> gpurun_out/$TAG/trace.err \
  || { echo "trace failed rc=$?"; tail -20 gpurun_out/$TAG/trace.err; exit 1; }
k=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"}; do
  k=$((k+1))
  echo "== pmc pass $k: $grp"
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/$TAG/pass$k -o run --output-format csv -- \
    python3 -u bench.py $ARGS --warmup 0 > gpurun_out/$TAG/pass$k.json 2> gpurun_out/$TAG/pass$k.err \
    || { echo "pass $k failed rc=$?"; tail -20 gpurun_out/$TAG/pass$k.err; exit 1; }
done
echo done
