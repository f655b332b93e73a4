set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./avrecode_amd/recode compress tests/fixtures/cockatoo.mp4 gpurun_out/c.avrc \
&& timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rdec -o run -- ./avrecode_amd/recode decompress gpurun_out/c.avrc gpurun_out/c.mp4 > gpurun_out/rdec.log 2>&1 \
&& cmp gpurun_out/c.mp4 tests/fixtures/cockatoo.mp4 && echo same \
&& AVR_LIBRARY=avrecode_amd/prof/libavrecode.so timeout -k 10 200 python scripts/prof_rmode.py > gpurun_out/prof_rmode.json 2>&1 \
&& cat gpurun_out/prof_rmode.json \
&& AVR_LIBRARY=avrecode_amd/prof/libavrecode.so timeout -k 10 200 python scripts/prof_sections.py --slices 1024 > gpurun_out/prof_par.json 2>&1 \
&& cat gpurun_out/prof_par.json
