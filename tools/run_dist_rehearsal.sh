#!/bin/bash
# GPU box (1 GPU): rehearse bench.py's N>1 control flow with 2 ranks sharing the card over the
# gloo backend (RCCL refuses two ranks on one device).  Topic replicas at the driver's default
# workload, then the filter-sharded layout (broadcast + gather + merge) on a smaller cfg3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dist
export EMQXGM_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 \
  > gpurun_out/dist/topics.json 2> gpurun_out/dist/topics.log
rc=$?; echo topics_exit=$rc; cat gpurun_out/dist/topics.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 3 --warmup 1 \
  --shard filters --filters 2000000 --topics 500000 \
  > gpurun_out/dist/filters.json 2> gpurun_out/dist/filters.log
rc=$?; echo filters_exit=$rc; cat gpurun_out/dist/filters.json; exit $rc
