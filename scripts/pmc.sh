#!/bin/bash
# PMC passes over a reduced bench run (one counter group per rocprofv3 pass, --kernel-trace only
# beside --pmc).  Output: gpurun_out/pmc_<tag>/pass<k>/..._counter_collection.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${PMC_ARGS:---slices 1024 --steps 1 --warmup 0 --no-cpu-baseline --no-files --no-corpus --no-p32}
mkdir -p gpurun_out/pmc_$TAG
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_$TAG/counters.txt 2>&1 || true
k=0
for grp in ${PMC_GROUPS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_IFETCH GRBM_GUI_ACTIVE" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_HITS" "FETCH_SIZE" "WRITE_SIZE"}; do
  k=$((k+1))
  echo "== pass $k: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$TAG/pass$k -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_$TAG/pass$k.json 2> gpurun_out/pmc_$TAG/pass$k.err || { echo "pass $k failed rc=$?"; tail -5 gpurun_out/pmc_$TAG/pass$k.err; exit 1; }
done
echo done
