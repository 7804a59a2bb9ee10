"""The multi-rank exchange in two processes on this box's one GPU: RCCL refuses two ranks on the same
device, so what runs here is the host-exchange transport -- the same per-step records moved over gloo
(np8_step_local / np8_step_merge).  (The RCCL code path itself runs in tests/test_gpu_rccl_one_rank.py with
a one-rank communicator; the driver's scaling runs use one GPU per rank.)  The sharded result must equal
the single-rank sweep bit for bit -- at N = 8000 from a poor start, at the C3 workload itself (N = 1e6, D = 8,
K = 64, warm state; the contiguous shards of C4) as 2, 4 and 8 ranks (8: the 125k-item shards of C4's 8-GPU point),
and from the reference's own initialisation at full size (init_random(20), 20 sweeps: the cold start's 158k requests
per step, partial acceptance by global scan position) as 2 ranks."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, D, SWEEPS, SEED = 8000, 8, 6, 2024
NC3, SWEEPS_C3 = 1_000_000, 12
SWEEPS_COLD = 20


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(kind="small"):
    from noparama_amd import datasets

    if kind == "cold":  # C3 data; the state comes from init_random(20) on every rank
        X, z, mu, sig = datasets.config_c3(N=NC3)
        return X, None, None, None
    if kind == "c3":  # the north-star workload: C3 data, its warm state (bench.py), 2% of the labels scrambled
        X, z, mu, sig = datasets.config_c3(N=NC3)
        z = z.astype(np.int32)
        rng = np.random.default_rng(3)
        idx = rng.choice(NC3, NC3 // 50, replace=False)
        z[idx] = rng.integers(0, mu.shape[0], size=idx.size)
        return X, z, mu, sig
    X, _, mu, sig = datasets.mixture(N, D, 10, 0.8, 8.0, seed=5)
    zr = np.random.default_rng(1).integers(0, 10, size=N).astype(np.int32)  # a poor start: many moves
    return X, zr, mu, sig


def _rank(rank, world, port, outdir, kind="small"):
    import torch
    import torch.distributed as dist

    from noparama_amd import NealAlgorithm8, NP8Error, comm_unique_id

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, zr, mu, sig = _data(kind)
    n, sweeps = X.shape[0], {"c3": SWEEPS_C3, "cold": SWEEPS_COLD}.get(kind, SWEEPS)
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
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
        smp.set_data(X[lo:hi], offset=lo, n_global=n)
        if kind == "cold":
            smp.init_random(20)
        else:
            smp.set_state(zr[lo:hi], mu, sig)
        smp.sweep(sweeps)
    else:
        transport = "gloo"
        smp.close()
        smp = NealAlgorithm8(D, seed=SEED, device=0)
        smp.comm_init(None, rank, world)
        smp.set_data(X[lo:hi], offset=lo, n_global=n)
        if kind == "cold":  # (init_random counts over all items: the global counts without communication)
            smp.init_random(20)
        else:
            smp.set_state(zr[lo:hi], mu, sig, counts=np.bincount(zr, minlength=mu.shape[0]))
        for _ in range(sweeps):
            rec = torch.from_numpy(smp.step_local())
            out = [torch.zeros_like(rec) for _ in range(world)]
            dist.all_gather(out, rec)
            smp.step_merge(np.concatenate([o.numpy() for o in out]), world)
            smp.end_sweep()
    st = smp.state()
    np.save(os.path.join(outdir, f"z{rank}.npy"), st["z"])
    np.save(os.path.join(outdir, f"c{rank}.npy"), st["counts"])
    np.save(os.path.join(outdir, f"k{rank}.npy"), np.array([st["K"], smp.stats()["rejected_requests"]]))
    open(os.path.join(outdir, f"transport{rank}"), "w").write(transport)
    dist.barrier()
    dist.destroy_process_group()


def _rank_compact(rank, world, port, outdir, cap):
    """The compact records of a sharded sweep graph over gloo: each step exchanges this rank's
    compact record (count deltas + the first `cap` requests); a step where some rank's requests do not fit halts
    alike on every rank and is resumed with the full records."""
    os.environ["NP8_COMPACT_REQ"] = str(cap)
    import torch
    import torch.distributed as dist

    from noparama_amd import NealAlgorithm8

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, _, _, _ = _data("cold")
    n = X.shape[0]
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
    smp = NealAlgorithm8(D, seed=SEED, device=0)
    smp.comm_init(None, rank, world)
    smp.set_data(X[lo:hi], offset=lo, n_global=n)
    smp.init_random(20)
    cb = smp.compact_record_bytes()
    assert cb > 0
    per_step = []  # (requests of every rank, halted)

    def all_gather(a):
        t = torch.from_numpy(a)
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        g = np.concatenate([o.numpy() for o in out])
        if a.size == cb:  # a compact record: its header's request count, per rank
            per_step.append([int(g[r * cb:r * cb + 4].view(np.int32)[0]) for r in range(world)])
        return g

    halts = 0
    for _ in range(SWEEPS_COLD):
        halts += smp.exchange_step(all_gather, world, compact=True)
        smp.end_sweep()
    st = smp.state()
    nreq = np.array(per_step)
    over = nreq > cap
    partial = int(np.sum(over.any(axis=1) & ~over.all(axis=1)))  # steps where only some ranks overflowed
    assert halts == int(np.sum(over.any(axis=1))) == smp.stats()["compact_halts"]
    np.save(os.path.join(outdir, f"z{rank}.npy"), st["z"])
    np.save(os.path.join(outdir, f"c{rank}.npy"), st["counts"])
    np.save(os.path.join(outdir, f"k{rank}.npy"),
            np.array([st["K"], smp.stats()["rejected_requests"], halts, partial]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cap", [(2, 1), (8, 1), (2, 32), (8, 32)])
def test_compact_records_gloo_cold_start_equals_single_rank(tmp_path, world, cap):
    """Compact records over the host transport from the reference's initialisation (init_random(20), C3 data,
    N = 1e6, 20 sweeps) at 2 and 8 ranks, capacity 1 and 32: the first steps overflow on every rank (halt, full
    records), the mixed regime's steps overflow on some ranks only; labels, counts, K and the rejected-request count
    equal one rank's (the full-record chain) bit for bit."""
    import torch.multiprocessing as mp

    from noparama_amd import NealAlgorithm8

    X, _, _, _ = _data("cold")
    one = NealAlgorithm8(D, seed=SEED, device=0)
    one.set_data(X)
    one.init_random(20)
    one.sweep(SWEEPS_COLD)
    ref = one.state()
    rej = one.stats()["rejected_requests"]
    one.close()
    mp.spawn(_rank_compact, args=(world, _port(), str(tmp_path), cap), nprocs=world, join=True)
    zz = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(world)])
    assert np.array_equal(zz, ref["z"])
    ks = [np.load(tmp_path / f"k{r}.npy") for r in range(world)]
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"c{r}.npy"), ref["counts"])
        assert list(ks[r][:2]) == [ref["K"], rej]
        assert list(ks[r][2:]) == list(ks[0][2:])  # halts and their kind alike on every rank
    halts, partial = int(ks[0][2]), int(ks[0][3])
    print(f"world {world} cap {cap}: {halts} halted steps of {SWEEPS_COLD}, {partial} with only some ranks over")
    assert 0 < halts < SWEEPS_COLD  # the first steps halt, the warm ones fit
    if cap == 1:
        assert partial > 0


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


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c3_workload_sharded_equals_single_rank(tmp_path, world):
    """C4's sharding of the C3 workload (N = 1e6, the warm state with 2% of the labels scrambled so that items move,
    contiguous shards) on 2, 4 and 8 ranks: labels and counts after 12 sweeps equal one rank's bit for bit."""
    import torch.multiprocessing as mp

    from noparama_amd import NealAlgorithm8

    X, z, mu, sig = _data("c3")
    one = NealAlgorithm8(D, seed=SEED, device=0)
    one.set_data(X)
    one.set_state(z, mu, sig)
    one.sweep(SWEEPS_C3)
    ref = one.state()
    one.close()
    mp.spawn(_rank, args=(world, _port(), str(tmp_path), "c3"), nprocs=world, join=True)
    zz = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(world)])
    assert np.array_equal(zz, ref["z"])
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"c{r}.npy"), ref["counts"])


def test_cold_start_full_size_sharded_equals_single_rank(tmp_path):
    """The reference's initialisation (np_mcmc.cpp:49-92: init_random(20)) at the full C3 size on 2 ranks, 20 sweeps:
    the first steps carry far more new-cluster requests than req_max (partial acceptance by global scan position,
    each rank sending its req_max lowest), later ones the mixed regime; labels, counts, K and the rejected-request
    count equal one rank's bit for bit."""
    import torch.multiprocessing as mp

    from noparama_amd import NealAlgorithm8

    X, _, _, _ = _data("cold")
    one = NealAlgorithm8(D, seed=SEED, device=0)
    one.set_data(X)
    one.init_random(20)
    one.sweep(SWEEPS_COLD)
    ref = one.state()
    rej = one.stats()["rejected_requests"]
    one.close()
    assert rej > 0  # the first step overflowed req_max
    mp.spawn(_rank, args=(2, _port(), str(tmp_path), "cold"), nprocs=2, join=True)
    zz = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(2)])
    assert np.array_equal(zz, ref["z"])
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"c{r}.npy"), ref["counts"])
        assert list(np.load(tmp_path / f"k{r}.npy")) == [ref["K"], rej]
