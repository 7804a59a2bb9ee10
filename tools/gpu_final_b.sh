#!/bin/bash
# One GPU call: the C4 shard budget (tools/c4_budget.sh) and the weak-scaling launch line rehearsed with two
# ranks on the one GPU (RCCL refuses two ranks on one device: the records go over gloo, "exchange": "gloo").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
bash tools/c4_budget.sh > gpurun_out/c4/summary.txt 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --weak --n 200000 --steps 20 --warmup 5 > gpurun_out/c4/weak_n2.json 2> gpurun_out/c4/weak_n2.err &&
echo FINAL_B_DONE
