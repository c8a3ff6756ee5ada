set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --rdzv-backend c10d --rdzv-endpoint 127.0.0.1:0 --rdzv-id probe --local-addr 127.0.0.1 tools/debug/rccl_two_ranks_one_gpu.py > gpurun_out/rccl2.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/rccl2.log | tail -20
