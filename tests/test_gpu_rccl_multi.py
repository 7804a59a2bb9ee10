"""The RCCL exchange with two ranks on two GPUs (skipped on a one-GPU box; the driver's 8-GPU node runs the same code
in bench.py): sharded sweep graphs whose compact records overflow (NP8_COMPACT_REQ=1 from init_random(20)), halts
resumed inside np8_sweep on every rank alike, then a rank-0-only statistics / state read -- which must not block,
since np8_sweep returns settled.  Labels, counts and K equal one rank's."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, D, SEED = 200_000, 8, 91


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, outdir):
    os.environ["NP8_COMPACT_REQ"] = "1"
    import torch.distributed as dist

    from noparama_amd import NealAlgorithm8, comm_unique_id, datasets

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, _, _, _ = datasets.mixture(N, D, 32, 0.8, 12.0, seed=9)
    lo, hi = (N * rank) // world, (N * (rank + 1)) // world
    uid = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    smp = NealAlgorithm8(D, seed=SEED, device=rank)
    smp.comm_init(uid[0], rank, world)
    smp.set_data(X[lo:hi], offset=lo, n_global=N)
    smp.init_random(20)
    for n in (20, 3, 40, 20):
        smp.sweep(n, sync=False)
        if rank == 0:  # one rank alone reads: no collective may be left for it to run
            smp.stats()
    st = smp.state()
    np.save(os.path.join(outdir, f"z{rank}.npy"), st["z"])
    np.save(os.path.join(outdir, f"k{rank}.npy"), np.array([st["K"], smp.stats()["compact_halts"]]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_gpu_rccl_compact_halts_equal_single_rank(tmp_path):
    import torch
    import torch.multiprocessing as mp

    from noparama_amd import NealAlgorithm8, datasets

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    X, _, _, _ = datasets.mixture(N, D, 32, 0.8, 12.0, seed=9)
    one = NealAlgorithm8(D, seed=SEED, device=0)
    one.set_data(X)
    one.init_random(20)
    one.sweep(83)
    ref = one.state()
    one.close()
    mp.spawn(_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    z = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(2)])
    assert np.array_equal(z, ref["z"])
    k = [np.load(tmp_path / f"k{r}.npy") for r in range(2)]
    assert int(k[0][0]) == int(k[1][0]) == ref["K"]
    assert int(k[0][1]) == int(k[1][1]) > 0
