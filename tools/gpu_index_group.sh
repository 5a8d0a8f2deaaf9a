set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or seed or golden or driver" > gpurun_out/idx_tests.log 2>&1 || { tail -30 gpurun_out/idx_tests.log; exit 1; }
tail -3 gpurun_out/idx_tests.log
for b in 1 0 1 0; do OVL_FINE_BITONIC=$b timeout -k 10 200 python tools/index_ab.py --reps 6 2>&1 | grep -v amdgpu.ids | sed "s/^/bitonic=$b /" || exit 1; done
