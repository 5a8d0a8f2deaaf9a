set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/diff_w5.py > gpurun_out/det.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/det.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
bash tools/g4.sh
