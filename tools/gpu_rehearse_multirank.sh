# multi-rank rehearsal on the 1-GPU box: 2 ranks share device 0 over gloo
set -o pipefail
mkdir -p gpurun_out
export CANU_DEVICE=0 CANU_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --reads 8000 --steps 1 --warmup 1 > gpurun_out/rh_ovl.log 2>&1 || { tail -30 gpurun_out/rh_ovl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rh_ovl.log | grep metric | cut -c1-600
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench_mhap.py --gpus 2 --reads 8000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/rh_mhap.log 2>&1 || { tail -30 gpurun_out/rh_mhap.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rh_mhap.log | grep metric | cut -c1-600
timeout -k 10 300 python bench.py --reads 8000 --steps 1 --warmup 1 --no-cpu-baseline | cut -c1-400
timeout -k 10 300 python bench_mhap.py --reads 8000 --steps 1 --warmup 1 --no-cpu-baseline | cut -c1-400
