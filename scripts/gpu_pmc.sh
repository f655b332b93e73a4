#!/bin/bash
# PMC evidence for the working build: HBM traffic and SQ instruction-mix passes (scripts/pmc.sh),
# then the summaries bench.py and DESIGN read: profiles/<RND>_pmc.json (with the build's
# source_sha) and gpurun_out/<TAG>_sq_counters.json.   gpurun -- 'TAG=r04i bash scripts/gpu_pmc.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r04i}
RND=${RND:-r04}
mkdir -p gpurun_out
TAG=$TAG bash scripts/pmc.sh \
&& python scripts/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/${RND}_pmc.json --slices 1024 --mb 120 68 > gpurun_out/pmc_traffic_$TAG.log \
&& python scripts/pmc_sq.py gpurun_out/pmc_$TAG gpurun_out/${TAG}_sq_counters.json --bins 2511192484 > gpurun_out/pmc_sq_$TAG.log \
&& cat gpurun_out/pmc_traffic_$TAG.log gpurun_out/pmc_sq_$TAG.log
