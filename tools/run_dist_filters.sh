#!/bin/bash
# GPU box (1 GPU): the N=2 filter-sharded layout as the headline (`--shard filters`), two ranks
# sharing the card over gloo (see tools/run_dist_rehearsal.sh: the timings mean nothing, the run
# shows the north-star layout reaching a bench line at the full cfg3 size)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dist_filters}
mkdir -p $O
export EMQXGM_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --shard filters --steps 5 --warmup 1 \
  > $O/n2.json 2> $O/n2.log
rc=$?; echo n2_exit=$rc; exit $rc
