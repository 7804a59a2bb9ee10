"""The multi-GPU exchange protocol on CPU with torch.distributed/gloo, world_size 2.

Each rank owns a contiguous shard of the items and a replica of the cluster table.  Per sweep it
evaluates its shard against the frozen state, all-gathers its exchange record (count deltas + new-
cluster requests with their global scan positions) and applies all records in rank order -- the
protocol np8_sweep runs over RCCL.  Here the per-rank compute is the oracle (this tests the protocol,
not the kernels; the GPU side of the same protocol is tests/test_gpu_parity.py::
test_host_exchange_two_ranks_equals_one).  The sharded result must equal the single-process sweep
bit for bit."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from noparama_amd import datasets

N, D, SWEEPS, SEED, KCAP = 3000, 3, 5, 31, 2048
REQ_MAX = 64  # small: the first sweeps from init_random defer most requests (partial acceptance)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, X, outdir):
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = (N * rank) // world, (N * (rank + 1)) // world
    c = O.Chain(D, seed=SEED, kcap=KCAP, req_max=REQ_MAX)
    c.set_data(X)  # replica of the data: only [lo, hi) is evaluated or owned
    c.init_random(20)
    codes = []
    for _ in range(SWEEPS):
        delta, rp, ri, rm, rz, n = c.assign_range(lo, hi)
        rec = [delta, rp, ri, rm, rz, n]
        allrec = [None] * world
        dist.all_gather_object(allrec, rec)
        dsum = np.sum([r[0] for r in allrec], axis=0).astype(np.int32)
        cat = [np.concatenate([r[k] for r in allrec]) for k in (1, 2, 3, 4)]
        codes.append(c.finalize(dsum, *cat, n_req=int(sum(r[5] for r in allrec)), owner_lo=lo, owner_hi=hi))
        c.end_sweep()
    z = c.state()["z"]
    np.save(os.path.join(outdir, f"z{rank}.npy"), z[lo:hi])
    np.save(os.path.join(outdir, f"k{rank}.npy"), np.array([c.K] + codes + list(c.request_stats)))
    dist.destroy_process_group()


def test_two_rank_gloo_sweeps_equal_single_process(tmp_path):
    import oracle as O

    X, _, _, _ = datasets.mixture(N, D, 8, 0.6, 4.0, seed=3)
    one = O.Chain(D, seed=SEED, kcap=KCAP, req_max=REQ_MAX)
    one.set_data(X)
    one.init_random(20)
    deferred = []
    for _ in range(SWEEPS):
        before = one.request_stats[1]
        assert one.sweep(1) == 0
        deferred.append(int(one.request_stats[1] - before))
    assert deferred[0] > 0  # the protocol's partial acceptance is exercised
    ref = one.state()
    mp.spawn(_rank, args=(2, _free_port(), X, str(tmp_path)), nprocs=2, join=True)
    z = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(2)])
    assert np.array_equal(z, ref["z"])
    for r in range(2):
        k = np.load(tmp_path / f"k{r}.npy")
        assert int(k[0]) == ref["K"] and list(k[1:1 + SWEEPS]) == deferred
        assert list(k[1 + SWEEPS:]) == list(one.request_stats)


CAP = 2  # compact records: room for this many requests per rank (NP8_COMPACT_REQ)


def _rank_compact(rank, world, port, X, outdir):
    """The compact-record form of the exchange:
    each rank gathers its count deltas and at most CAP requests with its request count; when some rank's count
    exceeds CAP -- seen alike by every rank in the gathered headers -- nothing is applied and the step is exchanged
    again with the full records."""
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = (N * rank) // world, (N * (rank + 1)) // world
    c = O.Chain(D, seed=SEED, kcap=KCAP, req_max=REQ_MAX)
    c.set_data(X)
    c.init_random(20)
    halts, partial = 0, 0
    for _ in range(SWEEPS):
        delta, rp, ri, rm, rz, n = c.assign_range(lo, hi)
        heads = [None] * world
        dist.all_gather_object(heads, [delta, rp[:CAP], ri[:CAP], rm[:CAP], rz[:CAP], n])
        over = [h[5] > CAP for h in heads]
        if any(over):  # halt: the full records of the same step
            halts += 1
            partial += not all(over)
            heads = [None] * world
            dist.all_gather_object(heads, [delta, rp, ri, rm, rz, n])
        dsum = np.sum([h[0] for h in heads], axis=0).astype(np.int32)
        cat = [np.concatenate([h[k] for h in heads]) for k in (1, 2, 3, 4)]
        c.finalize(dsum, *cat, n_req=int(sum(h[5] for h in heads)), owner_lo=lo, owner_hi=hi)
        c.end_sweep()
    np.save(os.path.join(outdir, f"z{rank}.npy"), c.state()["z"][lo:hi])
    np.save(os.path.join(outdir, f"k{rank}.npy"), np.array([c.K, halts, partial] + list(c.request_stats)))
    dist.destroy_process_group()


def test_two_rank_gloo_compact_records_equal_single_process(tmp_path):
    import oracle as O

    X, _, _, _ = datasets.mixture(N, D, 8, 0.6, 4.0, seed=3)
    one = O.Chain(D, seed=SEED, kcap=KCAP, req_max=REQ_MAX)
    one.set_data(X)
    one.init_random(20)
    for _ in range(SWEEPS):
        assert one.sweep(1) == 0
    ref = one.state()
    mp.spawn(_rank_compact, args=(2, _free_port(), X, str(tmp_path)), nprocs=2, join=True)
    z = np.concatenate([np.load(tmp_path / f"z{r}.npy") for r in range(2)])
    assert np.array_equal(z, ref["z"])
    k0 = np.load(tmp_path / "k0.npy")
    assert np.array_equal(k0, np.load(tmp_path / "k1.npy"))
    assert int(k0[0]) == ref["K"] and list(k0[3:]) == list(one.request_stats)
    assert 0 < int(k0[1]) <= SWEEPS  # the first steps from init_random(20) overflow the compact records
