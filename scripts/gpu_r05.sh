#!/bin/bash
# Round-5 evidence on one MI355X: rocprofv3 kernel stats of a reduced bench run (the headline
# batch only), then the PMC passes (scripts/pmc.sh: HBM traffic + SQ instruction mix) and their
# summaries.   gpurun -- 'TAG=r05l bash scripts/gpu_r05.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r05l}
RND=${RND:-r05}
mkdir -p gpurun_out/stats_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_$TAG -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-files --no-corpus --no-cpu-baseline --no-p32 \
  > gpurun_out/stats_$TAG/bench.json 2> gpurun_out/stats_$TAG/bench.err \
&& TAG=$TAG bash scripts/pmc.sh > gpurun_out/pmc_$TAG.log 2>&1 \
&& python scripts/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/${RND}_pmc.json --slices 1024 --mb 120 68 > gpurun_out/pmc_traffic_$TAG.log \
&& python scripts/pmc_sq.py gpurun_out/pmc_$TAG gpurun_out/${TAG}_sq_counters.json --bins 2511192484 > gpurun_out/pmc_sq_$TAG.log \
&& find gpurun_out/stats_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \; \
&& echo ok
