#!/bin/bash
# r03: the distributed / batcher GPU tests, the default bench line (NIF window sweep), then the
# N=2 rehearsal of the driver's multi-GPU command (gloo, two ranks on this box's one GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_dist}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_batcher.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
EMQXGM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 --topics 2000000 \
  > $O/n2.json 2> $O/n2.log || exit 1
