#!/bin/bash
# A/B of the headline step: the fused roundtrip kernel against the chain's four launches (same
# build, interleaved runs), then the GPU parity tests that run the fused path.  Output under
# gpurun_out/<TAG>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_fused}
mkdir -p gpurun_out/$TAG
A="--steps ${STEPS_N:-5} --warmup 1 --no-cpu-baseline --no-files --no-corpus --stream-leg-seconds 0"
for rep in 1 2; do
  for mode in fused fourlaunch; do
    extra=""; [ $mode = fourlaunch ] && extra="--no-fused"
    echo "== $mode $rep"
    timeout -k 10 300 python3 -u bench.py $A $extra > gpurun_out/$TAG/${mode}_$rep.json 2> gpurun_out/$TAG/${mode}_$rep.err \
      || { echo "$mode failed rc=$?"; tail -20 gpurun_out/$TAG/${mode}_$rep.err; exit 1; }
    python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=l['config'];print(round(l['value'],2),l['ms_per_step'],c.get('roundtrip_kernel_ms'),c.get('compress_ms'),c.get('decompress_ms'),l['bit_exact'],l.get('oracle_parity',{}).get('match'),l.get('p32',{}).get('value'))" gpurun_out/$TAG/${mode}_$rep.json
  done
done
if [ -n "$TESTS" ]; then
  echo "== tests $TESTS"
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/$TAG/tests.log; exit 1; }
  tail -3 gpurun_out/$TAG/tests.log
fi
echo done
