#!/bin/bash
# Extra bench legs: the configs[4] corpus (with a small configs[2] batch) and the configs[3]
# stream-shard mode at N=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== corpus" && timeout -k 10 600 python bench.py --slices 96 --steps 1 --warmup 1 --cpu-seconds 3 --no-files ${CORPUS_ARGS:-} > gpurun_out/bench_corpus.json 2> gpurun_out/bench_corpus.err \
&& cat gpurun_out/bench_corpus.json \
&& echo "== stream shard" && timeout -k 10 600 python bench.py --stream-shard --stream-seconds ${STREAM_SECONDS:-60} --steps 1 --warmup 1 > gpurun_out/bench_stream.json 2> gpurun_out/bench_stream.err \
&& cat gpurun_out/bench_stream.json
rc=$?
[ $rc -ne 0 ] && { tail -30 gpurun_out/bench_*.err 2>/dev/null; }
exit $rc
