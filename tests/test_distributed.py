"""Multi-process (world_size 2, gloo on CPU) checks of the sharding and the
deterministic cross-rank combination used for catchment sums and routing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shyft_amd import distributed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_covers_every_cell_once():
    for n in (1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 4, 8):
            ranges = [distributed.shard_range(n, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (b0, e0), (b1, e1) in zip(ranges, ranges[1:]):
                assert e0 == b1
            sizes = [e - b for b, e in ranges]
            assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # each rank owns a contiguous shard of per-cell series and reduces it locally
        n_cells, C, T = 101, 3, 17
        rng = np.random.default_rng(0)
        series = rng.normal(size=(T, n_cells))        # identical on every rank (same seed)
        cid = (np.arange(n_cells) * C) // n_cells
        b, e = distributed.shard_range(n_cells, world, rank)
        part = np.zeros((C, T))
        for c in range(C):
            sel = (cid[b:e] == c)
            part[c] = series[:, b:e][:, sel].sum(axis=1)
        total = distributed.combine_partials(torch.from_numpy(part)).numpy()
        t_max = distributed.max_over_ranks(float(rank + 1))
        q.put((rank, total, t_max))
    finally:
        dist.destroy_process_group()


class _FakeRegion:
    """CPU stand-in for HipRegion's routing-group interface (the per-rank device reduction)."""

    def __init__(self, q):
        self.q = q  # [T][n_local]

    def set_routing_groups(self, group_of_cell, n_groups):
        self.g, self.G = np.asarray(group_of_cell), n_groups

    def routing_group_sums(self, step0, n):
        out = np.zeros((self.G, n))
        for c in range(self.q.shape[1]):
            if self.g[c] >= 0:
                out[self.g[c]] += self.q[step0:step0 + n, c]
        return out


def _routing_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shyft_amd import synthetic
        n_total, T, C = 64, 12, 4
        series = np.random.default_rng(1).random((T, n_total))
        b, e = distributed.shard_range(n_total, world, rank)
        _, _, group = synthetic.cell_routing(e - b, C, cell_offset=b, n_total=n_total)
        sums = distributed.routing_group_sums(_FakeRegion(series[:, b:e]), group, C * 2, 0, T,
                                              device=torch.device("cpu")).numpy()
        q.put((rank, sums))
    finally:
        dist.destroy_process_group()


def test_routing_group_sums_gloo_world2():
    """Global (river, UHG) group sums from sharded cells equal the unsharded sums, identically on every rank."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_routing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1])
    from shyft_amd import synthetic
    n_total, T, C = 64, 12, 4
    series = np.random.default_rng(1).random((T, n_total))
    _, _, group = synthetic.cell_routing(n_total, C, n_total=n_total)
    ref = np.stack([series[:, group == g].sum(axis=1) for g in range(2 * C)])
    assert np.allclose(res[0][1], ref, rtol=1e-13, atol=1e-14)


def test_combine_partials_gloo_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    # identical on every rank, bitwise
    assert np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2] == 2.0
    # and equal to the single-process per-catchment sum
    n_cells, C, T = 101, 3, 17
    series = np.random.default_rng(0).normal(size=(T, n_cells))
    cid = (np.arange(n_cells) * C) // n_cells
    ref = np.stack([series[:, cid == c].sum(axis=1) for c in range(C)])
    assert np.allclose(res[0][1], ref, rtol=1e-13, atol=1e-13)


def _verify_worker(rank, world, port, inject_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = distributed.verify_collectives(inject_failure=(rank == inject_rank))
        host = distributed._COMBINE["host"]
        part = torch.from_numpy(np.arange(6, dtype=np.float64).reshape(2, 3) * (rank + 1))
        total = distributed.combine_partials(part).numpy()
        q.put((rank, rep, host, total, distributed.max_over_ranks(float(rank))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("inject_rank", [-1, 1])
def test_collective_self_check_and_host_fallback_gloo_world2(inject_rank):
    """verify_collectives: the known-value all-gather passes (no injection), or one rank's failure switches EVERY
    rank to the host path (they agree over the host backend); the combines give the same sums either way."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, inject_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rep, host, total, mx in res:
        assert host == (inject_rank >= 0), rep
        assert ("self-check passed" in rep) == (inject_rank < 0)
        assert np.array_equal(total, np.arange(6, dtype=np.float64).reshape(2, 3) * 3)
        assert mx == 1.0
    if inject_rank >= 0:
        assert "injected" in res[inject_rank][1] and "another rank" in res[1 - inject_rank][1]


@pytest.mark.gpu
def test_mixed_backend_group_on_the_gpu_box():
    """bench.py's rank group is "cpu:gloo,cuda:nccl": device tensors over RCCL, host tensors (the self-check's vote
    and the fallback combines) over gloo. One rank here (RCCL puts one rank per GPU): the group forms, a device
    all-gather and a host all-reduce both run, and the self-check reports."""
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("cpu:gloo,cuda:nccl", rank=0, world_size=1)
    try:
        dev = torch.device("cuda", 0)
        t = distributed._known(0, 64).to(dev)
        parts = [torch.empty_like(t)]
        dist.all_gather(parts, t)
        assert torch.equal(parts[0].cpu().view(torch.int64), distributed._known(0, 64).view(torch.int64))
        h = torch.tensor([3], dtype=torch.int64)
        dist.all_reduce(h, op=dist.ReduceOp.MIN)
        assert int(h.item()) == 3
        assert "single rank" in distributed.verify_collectives(device=dev)
        total = distributed.combine_partials(torch.ones(4, dtype=torch.float64, device=dev))
        assert total.is_cuda and float(total.sum()) == 4.0
    finally:
        dist.destroy_process_group()
