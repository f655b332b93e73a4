#!/bin/bash
# Reference-model compress of the fixtures: parallel pipeline vs the sequential kernel
# (AVR_RMODE_SEQUENTIAL=1); outputs must be identical.  Writes gpurun_out/rmode_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in realshort cockatoo; do
  for v in par seq; do
    if [ $v = seq ]; then export AVR_RMODE_SEQUENTIAL=1; else unset AVR_RMODE_SEQUENTIAL; fi
    s=$EPOCHREALTIME
    timeout -k 10 300 ./avrecode_amd/recode compress tests/fixtures/$f.mp4 gpurun_out/rmode_${f}_$v.avrc || exit 1
    e=$EPOCHREALTIME
    echo "$f $v $(awk "BEGIN{print $e - $s}") s $(sha256sum gpurun_out/rmode_${f}_$v.avrc | cut -c1-16)"
  done
  cmp gpurun_out/rmode_${f}_par.avrc gpurun_out/rmode_${f}_seq.avrc && echo "$f identical"
done
