"""Multi-GPU plumbing: one process per GPU, cells sharded in contiguous ranges.

run_cells has no cross-cell coupling (core/region_model.h:972-1021), so ranks
never exchange data while the cells run. The only exchanges are where the
reference itself aggregates over cells:
  - catchment sums / averages (cell_statistics, core/cell_model.h:228-368;
    region_model::catchment_discharges, core/region_model.h:873-885),
  - river local inflow for routing (core/routing.h:344-383).
Each rank reduces its own cells on its GPU into a small [C][T] partial; the
partials are all-gathered (RCCL over xGMI with backend "nccl", gloo on CPU) and
summed in rank order on every rank, so the result is identical on all ranks
and run to run (no reduction-order nondeterminism).
"""
from __future__ import annotations

import os


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """[begin, end) of the cells owned by `rank` (contiguous, sizes differ by at most one)."""
    base, extra = divmod(n_total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def env_rank() -> tuple[int, int, int]:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


# set by verify_collectives: the device collectives failed their self-check (or raised), so every later combine
# moves its (small) partials through the host backend of the same process group instead
_COMBINE = {"host": False, "report": "not verified"}


def _wire(t, group=None):
    """The tensor the backend can move: RCCL ("nccl") takes device tensors; gloo (the CPU rehearsal
    backend, also used for more ranks than GPUs on one box, and the fallback after a failed RCCL self-check)
    only host tensors."""
    import torch.distributed as dist
    if t.is_cuda and (_COMBINE["host"] or dist.get_backend(group) == "gloo"):
        return t.cpu()
    return t


def _known(rank: int, m: int):
    """m doubles that depend on the rank, signed, spread over 60 binades (every mantissa bit matters)"""
    import torch
    j = torch.arange(m, dtype=torch.int64)
    mant = ((rank * 2654435761 + j * 40503) % 1000003).to(torch.float64) + 0.5
    mant = torch.where(j % 2 == 1, -mant, mant)
    return torch.ldexp(mant, (j % 61 - 30).to(torch.float64))


def verify_collectives(device=None, group=None, inject_failure: bool = False, m: int = 4096) -> str:
    """Bit-exact self-check of the all-gather the combines use, before any data goes through it: every rank
    contributes m known doubles, every rank must receive all of them bit for bit. The ranks agree on the outcome
    over the host backend (a CPU all-reduce of a flag); if any rank failed (or the collective raised), every later
    combine_partials / max_over_ranks moves its partials through the host backend instead -- the same values,
    slower. With a mixed process group ("cpu:gloo,cuda:nccl") that host path needs no second group; a group with no
    host backend (RCCL alone) has no such path, and a failed self-check raises there instead. Returns the report
    (also in combine_report()). inject_failure: the fallback test's failure on this rank."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        _COMBINE.update(host=False, report="single rank: nothing to combine")
        return _COMBINE["report"]
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    ok, why = True, ""
    # the tensors are built before the collective, and every rank enters the all-gather exactly once whatever fails
    # on it (a rank that skipped it would leave the others blocked in it)
    try:
        t = _known(rank, m)
        if device is not None:
            t = t.to(device)
        parts = [torch.empty_like(t) for _ in range(world)]
    except Exception as e:  # noqa: BLE001 -- preparation failed: take part with a dummy, report the failure
        ok, why = False, f"{type(e).__name__}: {e}"
        t = torch.zeros(m, dtype=torch.float64, device=device if device is not None else "cpu")
        parts = [torch.empty_like(t) for _ in range(world)]
    try:
        dist.all_gather(parts, t, group=group)
        if inject_failure:
            raise RuntimeError("injected all-gather failure")
        for r in range(world) if ok else ():
            got = parts[r].cpu().view(torch.int64)
            if not torch.equal(got, _known(r, m).view(torch.int64)):
                ok, why = False, f"rank {rank} received rank {r}'s values with different bits"
                break
    except Exception as e:  # noqa: BLE001 -- any failure of the device path means: use the host path
        ok, why = False, f"{type(e).__name__}: {e}"
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
    host_backend = "gloo" in str(dist.get_backend(group)) or device is None
    if host_backend:
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)   # host tensor: the group's CPU backend
    else:  # a device-only group: agree over the device (no host path to fall back to then)
        fd = flag.to(device)
        dist.all_reduce(fd, op=dist.ReduceOp.MIN, group=group)
        flag = fd.cpu()
    if int(flag.item()) == 1:
        kind = "device" if device is not None and getattr(device, "type", "cpu") == "cuda" else "host"
        _COMBINE.update(host=False, report=f"{kind} all-gather self-check passed ({world} ranks x {m} known doubles "
                                           f"bit-exact on every rank)")
    else:
        report = ("the device all-gather self-check failed" + (f" on this rank ({why})" if why else " on another rank"))
        if not host_backend:
            # a group without a CPU backend cannot move host tensors: no combine could work, say so now
            _COMBINE.update(host=False, report=report + "; no host backend in this process group")
            raise RuntimeError(_COMBINE["report"])
        _COMBINE.update(host=True, report="host (gloo) combines: " + report)
    return _COMBINE["report"]


def combine_report() -> str:
    return _COMBINE["report"]


def combine_partials(partial, group=None, out=None):
    """Deterministic cross-rank sum of per-rank partials (a torch tensor, same shape on every
    rank): all_gather, then add in rank order. Returns the total on every rank (written into
    `out` when given)."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        if out is None:
            return partial.clone()
        out.copy_(partial)
        return out
    world = dist.get_world_size(group)
    wire = _wire(partial.contiguous(), group)
    parts = [torch.empty_like(wire) for _ in range(world)]
    dist.all_gather(parts, wire, group=group)
    total = parts[0].clone()
    for p in parts[1:]:
        total += p
    if out is None:
        return total.to(partial.device)
    out.copy_(total)
    return out


def max_over_ranks(value: float, device=None, group=None) -> float:
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    t = _wire(torch.tensor([float(value)], dtype=torch.float64, device=device), group)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def routing_group_sums(region, local_groups, n_global_groups: int, step0: int, n: int, group=None, device=None):
    """Discharge sums of the global routing groups (cells sharing river + UHG, core/routing.h:326-345) over
    ALL ranks' cells. local_groups[n_local_cells] holds each local cell's global group index (-1 = not
    routed); the rank's group sums are formed on its GPU and combined in rank order (combine_partials).
    Returns a torch tensor [n_global_groups][n] on `device`, identical on every rank."""
    import torch
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    region.set_routing_groups(local_groups, n_global_groups)
    part = torch.empty((n_global_groups, n), dtype=torch.float64, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
        region.routing_group_sums_device(step0, n, part.data_ptr())
    else:
        part.copy_(torch.from_numpy(region.routing_group_sums(step0, n)))
    return combine_partials(part, group)


def catchment_sums(region, series: int, step0: int, n: int, global_cids, group=None, device=None):
    """Per-catchment sums of a response series over ALL ranks' cells.

    global_cids: the catchment ids of the whole region, in the order wanted for
    the result (e.g. the reference's cix order of the unsharded region). Each
    rank sums its own cells per local catchment on its GPU, places the rows at
    their global positions and the partials are combined in rank order.
    Returns a torch tensor [len(global_cids)][n] on `device`."""
    import torch
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    local = [int(c) for c in region.catchment_ids()]
    pos = {int(c): i for i, c in enumerate(global_cids)}
    missing = [c for c in local if c not in pos]
    if missing:
        raise RuntimeError(f"one or more supplied catchment_indexes does not exist:{missing[0]}")
    part = torch.empty((len(local), n), dtype=torch.float64, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
        region.catchment_sums_device(series, step0, n, part.data_ptr())
    else:
        part.copy_(torch.from_numpy(region.catchment_sums(series, step0, n)))
    full = torch.zeros((len(global_cids), n), dtype=torch.float64, device=dev)
    full[torch.tensor([pos[c] for c in local], device=dev, dtype=torch.long)] = part
    return combine_partials(full, group)
