#!/bin/bash
# One GPU call: the weak-scaling launch line rehearsed with two ranks on the one GPU (RCCL refuses two ranks on
# one device: the records go over gloo, "exchange": "gloo"; 10^6 items per rank), and a kernel trace of the C5
# sweep with the niw_conjugate parameter update.  (The C4 shard budget: tools/c4_budget.sh.)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --weak --steps 20 --warmup 5 > gpurun_out/c4/weak_n2.json 2> gpurun_out/c4/weak_n2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5conj -o run -- python3 bench.py --config C5 --param-update niw_conjugate --steps 10 --warmup 5 --cpu-seconds 0 > gpurun_out/c5conj.log 2>&1 &&
echo FINAL_B_DONE
