set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_files.py tests/test_gpu_cli.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_files.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" gpurun_out/pytest_files.log | tail -60; exit $rc
