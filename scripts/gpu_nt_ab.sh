#!/bin/bash
# A/B of builds (LIBS: name=path ...) on the configs[3] stream's HBM traffic (rocprofv3 FETCH_SIZE /
# WRITE_SIZE passes over a 60-s stream leg) and the headline batch's time (bench.py, 3 steps).
# Output under gpurun_out/<TAG>/<name>_*; each step under its own time limit, first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_ab}
SECS=${SECS:-60}
mkdir -p gpurun_out/$TAG
for spec in ${LIBS:-main=avrecode_amd/libavrecode.so}; do
  name=${spec%%=*}; lib=${spec#*=}
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $name $c"
    AVR_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/$TAG/${name}_$c -o run \
      --output-format csv -- python3 -u bench.py --stream-shard --stream-seconds $SECS --steps 1 --warmup 0 \
      > gpurun_out/$TAG/${name}_$c.json 2> gpurun_out/$TAG/${name}_$c.err \
      || { echo "$name $c failed rc=$?"; tail -20 gpurun_out/$TAG/${name}_$c.err; exit 1; }
  done
  for rep in ${REPS:-1}; do
    echo "== $name headline $rep"
    AVR_LIBRARY=$lib timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files \
      --no-corpus --no-p32 --stream-leg-seconds 0 > gpurun_out/$TAG/${name}_head$rep.json \
      2> gpurun_out/$TAG/${name}_head$rep.err \
      || { echo "$name headline failed rc=$?"; tail -20 gpurun_out/$TAG/${name}_head$rep.err; exit 1; }
    tail -c 400 gpurun_out/$TAG/${name}_head$rep.json
  done
done
echo done
