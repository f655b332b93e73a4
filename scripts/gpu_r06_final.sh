#!/bin/bash
# Round-6 end evidence on one frozen build, in parts that each fit one gpurun call (PART=a|b|c|d):
#   a  smoke + the whole -m gpu suite
#   b  the headline's PMC passes (HBM traffic, SQ instruction mix) -> gpurun_out/r06_pmc.json (the file
#      bench.py --round r06 reads), r06z_sq_counters.json; rocprofv3 kernel stats of a short headline run
#   c  configs[3]'s queue kernel on the 600-s stream: timed step, kernel stats, PMC passes
#      (scripts/gpu_stream_prof.sh) -> gpurun_out/r06_stream_pmc.json
#   d  the default bench line, and rocprofv3 kernel stats of the long-slice split on the 4K 4:4:4 file
# Each GPU step has its own time limit; the first failure ends the part.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
case ${PART:-a} in
  a)
    echo "== smoke" && timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    && tail -2 $O/smoke.log \
    && echo "== pytest -m gpu" \
    && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    && tail -3 $O/pytest_gpu.log ;;
  b)
    TAG=r06z bash scripts/pmc.sh \
    && python scripts/pmc_traffic.py gpurun_out/pmc_r06z gpurun_out/r06_pmc.json --slices 1024 --mb 120 68 > $O/pmc_traffic.log \
    && python scripts/pmc_sq.py gpurun_out/pmc_r06z gpurun_out/r06z_sq_counters.json --bins 2511192484 > $O/pmc_sq.log \
    && echo "== kernel stats" \
    && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
         python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-files --no-corpus --no-p32 --stream-leg-seconds 0 \
         > $O/bench_prof.json 2> $O/bench_prof.err \
    && tail -c 400 $O/bench_prof.json ;;
  c)
    TAG=r06z_stream bash scripts/gpu_stream_prof.sh \
    && python scripts/pmc_traffic.py gpurun_out/r06z_stream gpurun_out/r06_stream_pmc.json --leg stream_shard \
         --seconds 600 --mb 240 135 > $O/stream_pmc_traffic.log ;;
  d)
    echo "== bench" && timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err \
    && tail -c 600 $O/bench.json \
    && echo "== split kernel stats" \
    && PROBE_ONLY=4K_IBBP timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split_prof -o run -- \
         python3 -u scripts/long_slice_probe.py > $O/split_probe.json 2> $O/split_probe.err ;;
esac
