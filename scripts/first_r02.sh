set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in realshort cockatoo; do
  for m in "" "-p"; do
    echo "== $f $m"
    s=$EPOCHREALTIME
    timeout -k 10 120 ./avrecode_amd/recode roundtrip $m tests/fixtures/$f.mp4 gpurun_out/$f$m.avrc || { echo "FAILED rc=$?"; exit 1; }
    e=$EPOCHREALTIME; echo "wall $(awk "BEGIN{print $e - $s}")"
    sha256sum gpurun_out/$f$m.avrc
  done
done
echo "== pytest" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; tail -3 gpurun_out/pytest_gpu.log
