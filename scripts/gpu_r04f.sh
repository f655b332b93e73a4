#!/bin/bash
# Round 4: one session on the working build -- smoke, the whole -m gpu suite, the default bench and
# its rocprofv3 kernel stats (scripts/gpu_round.sh), then the walker section profile (AVR_PROFILE
# build) of the headline batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04f}
ROUND=$tag bash scripts/gpu_round.sh || exit $?
echo "== section profile" && AVR_LIBRARY=avrecode_amd/prof/libavrecode.so timeout -k 10 300 python scripts/prof_sections.py --slices 1024 > gpurun_out/${tag}_sections.json 2> gpurun_out/${tag}_sections.err
rc=$?
head -80 gpurun_out/${tag}_sections.json
exit $rc
