"""The multi-rank exchange in two processes on this box's one GPU: RCCL refuses two ranks on the same
device, so what runs here is the host-exchange transport -- the same per-step records moved over gloo
(np8_step_local / np8_step_merge).  (The RCCL code path itself runs in tests/test_gpu_rccl_one_rank.py with
a one-rank communicator; the driver's scaling runs use one GPU per rank.)  The sharded result must equal
the single-rank sweep bit for bit."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, D, SWEEPS, SEED = 8000, 8, 6, 2024


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from noparama_amd import datasets

    X, _, mu, sig = datasets.mixture(N, D, 10, 0.8, 8.0, seed=5)
    zr = np.random.default_rng(1).integers(0, 10, size=N).astype(np.int32)  # a poor start: many moves
    return X, zr, mu, sig


def _rank(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    from noparama_amd import NealAlgorithm8, NP8Error, comm_unique_id

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, zr, mu, sig = _data()
    lo, hi = (N * rank) // world, (N * (rank + 1)) // world
    uid = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    smp = NealAlgorithm8(D, seed=SEED, device=0)
    try:
        smp.comm_init(uid[0], rank, world)
        ok = True
    except NP8Error:
        ok = False
    flags = [None] * world
    dist.all_gather_object(flags, ok)
    if all(flags):
        transport = "rccl"
        smp.set_data(X[lo:hi], offset=lo, n_global=N)
        smp.set_state(zr[lo:hi], mu, sig)
        smp.sweep(SWEEPS)
    else:
        transport = "gloo"
        smp.close()
        smp = NealAlgorithm8(D, seed=SEED, device=0)
        smp.comm_init(None, rank, world)
        smp.set_data(X[lo:hi], offset=lo, n_global=N)
        smp.set_state(zr[lo:hi], mu, sig, counts=np.bincount(zr, minlength=mu.shape[0]))
        for _ in range(SWEEPS):
            rec = torch.from_numpy(smp.step_local())
            out = [torch.zeros_like(rec) for _ in range(world)]
            dist.all_gather(out, rec)
            smp.step_merge(np.concatenate([o.numpy() for o in out]), world)
            smp.end_sweep()
    st = smp.state()
    np.save(os.path.join(outdir, f"z{rank}.npy"), st["z"])
    np.save(os.path.join(outdir, f"c{rank}.npy"), st["counts"])
    open(os.path.join(outdir, f"transport{rank}"), "w").write(transport)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_processes_equal_single_rank(tmp_path):
    import torch.multiprocessing as mp

    from noparama_amd import NealAlgorithm8

    X, zr, mu, sig = _data()
    one = NealAlgorithm8(D, seed=SEED, device=0)
    one.set_data(X)
    one.set_state(zr, mu, sig)
    one.sweep(SWEEPS)
    ref = one.state()
    one.close()
    mp.spawn(_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    z = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(2)])
    assert np.array_equal(z, ref["z"])
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"c{r}.npy"), ref["counts"])
    print("transport:", open(tmp_path / "transport0").read())
