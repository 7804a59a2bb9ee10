#!/bin/bash
# The driver's 2-rank launch line on a one-GPU box (RCCL refuses two ranks on one device, so both ranks fall back to the
# gloo records; a launch-path check, not a scaling number).  Run on the GPU box from the repo root:
#   /usr/local/graft/bin/gpurun -- 'bash tools/n2_rehearsal.sh'
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/n2 && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/n2/bench.json 2> gpurun_out/n2/bench.err
rc=$?; echo "rc=$rc"; tail -c 600 gpurun_out/n2/bench.json; exit $rc
