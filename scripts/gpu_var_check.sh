#!/bin/bash
# Parity of experiment builds (avrecode_amd/var/<name>/libavrecode.so) on the decompress-side GPU
# tests, then an A/B timing of them against the working build:
#   gpurun -- 'bash scripts/gpu_var_check.sh <tag> <name> [<name> ...]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; shift
for name in "$@"; do
  echo "== parity ($name)"
  AVR_LIBRARY=avrecode_amd/var/$name/libavrecode.so LD_LIBRARY_PATH=$PWD/avrecode_amd/var/$name timeout -k 10 900 \
    python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_fields.py tests/test_gpu_clip.py tests/test_gpu_files.py tests/test_gpu_cli.py \
    > gpurun_out/${tag}_${name}_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${tag}_${name}_tests.log
  [ $rc -eq 0 ] || exit $rc
done
echo "== A/B" && bash scripts/gpu_ab_r04.sh $tag "$@"
