set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in realshort cockatoo; do
  for m in "" "-p"; do
    echo "== $f $m"
    timeout -k 10 120 ./avrecode_amd/recode roundtrip $m tests/fixtures/$f.mp4 gpurun_out/$f$m.avrc || { echo "FAILED rc=$?"; exit 1; }
    sha256sum gpurun_out/$f$m.avrc
  done
done
