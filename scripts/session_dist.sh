#!/bin/bash
# Two ranks of bench.py on one GPU over gloo: the N>1 code path (round-robin
# shards, barrier, max-over-ranks timing, rank-0 JSON) the driver runs over
# RCCL on 8 GPUs.
set -u
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
POM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu > gpurun_out/dist.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dist.log | tail -3; exit $rc
