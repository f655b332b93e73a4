#!/bin/bash
# Round-end evidence on one build: PMC passes (HBM traffic + SQ instruction mix, one counter group
# per rocprofv3 pass), the traffic summary bench.py reads (profiles/<round>_pmc.json, with the
# build's source_sha), then smoke, the -m gpu suite, the default bench and its rocprofv3 kernel
# stats.  Copies of every summary land in gpurun_out/.   gpurun -- 'TAG=r04z bash scripts/gpu_final.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r04z}
RND=${RND:-r04}   # profiles/<RND>_pmc.json: the file bench.py --round RND reads
mkdir -p gpurun_out
TAG=$TAG bash scripts/pmc.sh \
&& python scripts/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/${RND}_pmc.json --slices 1024 --mb 120 68 > gpurun_out/pmc_traffic_$TAG.log \
&& cp gpurun_out/${RND}_pmc.json profiles/${RND}_pmc.json \
&& python scripts/pmc_sq.py gpurun_out/pmc_$TAG gpurun_out/${TAG}_sq_counters.json --bins 2511192484 > gpurun_out/pmc_sq_$TAG.log \
&& ROUND=$TAG bash scripts/gpu_round.sh
