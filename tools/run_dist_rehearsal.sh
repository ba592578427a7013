#!/bin/bash
# GPU box (1 GPU): rehearse bench.py's N>1 path with 2 ranks sharing the card over the gloo
# backend (RCCL refuses two ranks on one device; gloo stages the messages through host memory).
# The driver's default N>1 command: replicas as `value`, the filter-sharded layout (broadcast,
# per-shard match + export, count all_gather, grouped send/recv to rank 0, emqxgm_merge) beside
# it, at the full cfg3 size (10M filters, 2M-topic batches).  The timings are two processes
# time-slicing one GPU and gloo's host staging; what the rehearsal shows is that the N>1 path
# runs to a bench line at full size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dist}
mkdir -p $O
export EMQXGM_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 \
  > $O/n2.json 2> $O/n2.log
rc=$?; echo n2_exit=$rc; cat $O/n2.json; exit $rc
