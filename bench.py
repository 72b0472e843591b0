#!/usr/bin/env python3
"""Headline benchmark: pt_gs_k region_model::run_cells cell-steps/s on MI355X.

Workload (BASELINE.json configs[1]): pt_gs_k, 1M synthetic cells per GPU x 8760
hourly steps, fp64. A bench "step" is one pass of the hot path over one batch:
all cells of the rank advanced through one chunk of CHUNK=438 hourly steps
(1/20 year) -- the chunk's forcing is generated into HBM by the device
generator and run_cells runs the pt_gs_k kernel over it, state
carried in HBM to the next chunk. --steps 20 (the default, and the driver's
command) therefore runs exactly configs[1]'s year: Jan 1 - Dec 31, 8760 steps.
The per-cell fp64 forcing of a full year (350 GB at 1M cells) does not fit
one GPU's 288 GB, hence the chunking; generating a chunk costs ~1% of the step
and is inside the timed region (conservative).

Multi-GPU (--gpus N, one process per GPU via torch.distributed.run): cells
shard with no data-path collective (run_cells has no cross-cell coupling,
region_model.h:972-1021), weak scaling: each rank owns 1M cells of an
N x 1M-cell region. Timing: barrier + synchronize around exactly K steps,
max over ranks.

--stack hbv_stack runs configs[3]'s stack (hbv_snow + hbv_soil + hbv_tank,
core/hbv_stack.h:278-361) on 512K cells per GPU, so that --gpus 8 is the
4M-cell C4 region.

Extra fields: roofline (dominant kernel = ptgsk_run_kernel, HBM-bound
accounting per SURVEY.md §8d, kernel time from HIP events on the region's
stream) and cpu_baseline (the CPU oracle built with the host libm, run with the
reference's scheduler -- use_ncore std::async workers pulling one cell per
mutex-protected pos++, region_model.h:991-1021 -- on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "cell-steps/sec (cells×timesteps/wall) for pt_gs_k at 1/2/4/8 MI355X"
CHUNK = 438                      # 20 chunks = one calendar year (8760 hourly steps)
YEAR = 8760
HBM_PEAK_BPS = 8.0e12            # MI355X HBM3E spec (MI355X_MICROARCH.md)
SMALL_REGION_CELLS = 2 * 256 * 256   # cells per GPU at which a 256-lane launch gives each CU at most 2 workgroups
# algorithmic HBM bytes of the dominant kernel
STACKS = {
    # name: (forcing bytes read per cell-step, series bytes written per cell-step, state bytes per cell per launch,
    #        kernel name)
    "pt_gs_k": (40, 16, 2 * 9 * 8, "ptgsk_run_kernel"),      # T P WS RH RAD in; discharge, charge out; 9 state
    "hbv_stack": (32, 16, 2 * 22 * 8, "hbv_run_kernel"),     # wind not read (hbv_stack.h:295-301); 22 state
    "pt_ss_k": (32, 16, 2 * 8 * 8, "ptssk_run_kernel"),      # T P RH RAD in (wind not read: skaugen does not use it); 8 state
    "pt_hs_k": (32, 16, 2 * 20 * 8, "pthsk_run_kernel"),     # T P RH RAD in (no wind: hbv_snow); 20 state (bins + q)
    "pt_hps_k": (40, 16, 2 * 37 * 8, "pthpsk_run_kernel"),   # T P WS RH RAD in; 37 state (hps bins + q)
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launch", choices=("engine", "ranks"), default=None,
                    help="--gpus N > 1 without an outside launcher: 'ranks' (the default) = start N rank processes "
                         "(one per GPU, torch.distributed), as torch.distributed.run does; 'engine' = this one process "
                         "drives the N GPUs through a sharded region (shyft_hip_region_create_sharded: one shard per "
                         "GPU, catchment / routing sums all-gathered by RCCL inside the engine after its self-check, "
                         "device copies if RCCL fails). --gpus 1 --shards S always runs the engine's shards")
    ap.add_argument("--shards", type=int, default=0,
                    help="engine path: shards of the region (default: one per GPU); more shards than GPUs share "
                         "devices round-robin (on one GPU: --gpus 1 --shards 2 runs two shards on device 0)")
    ap.add_argument("--balance-z", action="store_true",
                    help="engine shards dealt by elevation rank (SHYFT_HIP_SHARD_BALANCE_Z) instead of contiguous ranges")
    ap.add_argument("--steps", type=int, default=YEAR // CHUNK)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cells", type=int, default=0,
                    help="cells per GPU (default 1,048,576 for pt_gs_k, 524,288 for hbv_stack)")
    ap.add_argument("--total-cells", type=int, default=0,
                    help="strong scaling: a region of this many cells split over the ranks (shard_range) instead of "
                         "--cells per GPU")
    ap.add_argument("--catchments", type=int, default=0,
                    help="catchments of the whole region (default 100 per 1M-cell shard, 100 with --total-cells)")
    ap.add_argument("--no-catchment-sums", action="store_true",
                    help="skip the per-chunk catchment discharge sums (cell_statistics, RCCL allgather)")
    ap.add_argument("--dump-sums", default="",
                    help="rank 0 saves the region's catchment discharge sums [C][T] (.npy) after the timed steps")
    ap.add_argument("--dump-route", default="",
                    help="rank 0 saves the routed river series (local, upstream, output) [3][R][T] (.npy) after the "
                         "timed steps")
    ap.add_argument("--dist-check", action="store_true",
                    help="launcher/rendezvous/collective rehearsal without the GPU: every rank combines "
                         "catchment sums of a synthetic series over its shard, rank 0 checks them against "
                         "the unsharded sums (tests/test_bench_launch.py)")
    ap.add_argument("--stack", choices=tuple(STACKS), default="pt_gs_k")
    ap.add_argument("--routing", action="store_true",
                    help="configs[4]: route avg_discharge through the synthetic river network (routing::uhg): "
                         "per chunk the (river, UHG)-group sums are formed on each GPU and all-gathered, after the "
                         "last chunk the network is convolved on the device (on by default for --stack pt_ss_k)")
    ap.add_argument("--no-routing", action="store_true")
    ap.add_argument("--pipeline", action="store_true",
                    help="two regions: generate chunk s+1's forcing while chunk s runs (measured slower for pt_gs_k, "
                         "see DESIGN.md section 5; off by default)")
    ap.add_argument("--overlap-forcing", type=int, default=None, metavar="CUS",
                    help="generate chunk s+1's forcing into a second window buffer on a side stream while chunk s "
                         "runs: CUS > 0 CUs, or -1 the whole device at the lowest stream priority (0: generate each "
                         "chunk before its run). Default: -1 for a region too small to fill the GPU (<= 131,072 "
                         "cells per GPU), else 0")
    ap.add_argument("--chunk", type=int, default=CHUNK)
    ap.add_argument("--cpu-cells", type=int, default=4000, help="cpu_baseline sample cells (x 8760 steps)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, os cpu share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--idw", action="store_true",
                    help="configs[2]: forcing interpolated each chunk by IDW from 500 stations (run_interpolation) "
                         "instead of the per-cell generator")
    ap.add_argument("--btk", action="store_true",
                    help="as --idw, but temperature by Bayesian kriging from the stations (the reference's default "
                         "temperature method, region_model.h:460-468)")
    return ap.parse_args(argv)


# configs[2] station network: 500 stations on a 22 x 23 grid at 45 km spacing
# covering the cell region, z in [0, 2000) m, values from the same generator (station ids offset by 2^40)
N_STATIONS = 500
STATION_ID0 = 1 << 40


def station_network(world_cells):
    from shyft_amd import synthetic
    import math
    W = int(math.ceil(math.sqrt(world_cells)))
    span = W * 1000.0
    k = np.arange(N_STATIONS)
    gx, gy = 22, 23
    xyz = np.zeros((N_STATIONS, 3))
    xyz[:, 0] = (k % gx) * (span / (gx - 1))
    xyz[:, 1] = (k // gx) * (span / (gy - 1))
    xyz[:, 2] = synthetic.elevation(N_STATIONS, synthetic.SEED, STATION_ID0)
    return xyz


def station_values(xyz, step0, n):
    from shyft_amd import synthetic
    f = synthetic.forcing(N_STATIONS, step0, n, synthetic.SEED, cell_offset=STATION_ID0, z=xyz[:, 2])
    return f  # [5][n][S]


# IDW parameters in the C ABI layout: max_members, max_distance, f, zscale, default gradient,
# gradient_by_equation, precipitation scale (inverse_distance.h:38-74 defaults)
IDW_DEFAULTS = {
    0: [20, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],   # temperature_parameter
    1: [20, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],   # precipitation_parameter
    2: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],   # wind_speed (parameter)
    3: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],   # rel_hum
    4: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],   # radiation
}


def idw_gather_bytes(var, cells, rows, n_sources=N_STATIONS):
    """Algorithmic HBM bytes of one IDW gather launch (kernels/idw.hip, wavefront-union path) for forcing variable
    `var` over `rows` steps: the window rows it writes (8 B per cell-step) plus what it reads once per launch -- per
    cell the neighbour table (K packed 1-byte local indexes, K weights, and for temperature / precipitation K
    transform terms: d.z - s.z or pow(scale, dz/100)), its member count, the cell's z (temperature) or slope
    (radiation), its wavefront's share of the union list (64 x 4 B per 64 cells), and the [rows][sources] values."""
    K = int(IDW_DEFAULTS[var][0])
    per_cell = K * (1 + 8 + (8 if var in (0, 1) else 0)) + 4 + 4 + (8 if var in (0, 4) else 0)
    return cells * rows * 8 + cells * per_cell + rows * n_sources * 8


# bayesian_kriging::parameter() defaults (bayesian_kriging.h:204-217) in the C ABI layout:
# gradient_sd [C/m], sill, nugget, range, zscale
BTK_DEFAULTS = [0.0025, 25.0, 0.5, 200000.0, 20.0]
FP64_PEAK_FLOPS = 78.6e12        # MI355X FP64 matrix/vector peak (AMD spec sheet; not in MI355X_MICROARCH.md)


def launch_ranks(n_gpus):
    """`bench.py --gpus N` started without a launcher: this parent process starts N fresh rank processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, 127.0.0.1 rendezvous) and exits with the first
    failing rank's status. Each rank is a supervisor (shyft_amd/supervise.py) that runs the real rank as its child and
    falls back from RCCL to gloo combines if an attempt fails or stalls; the parent never touches the GPU and, as a last
    resort, ends everything at a wall deadline (SHYFT_LAUNCH_DEADLINE_S, default 3600 s)."""
    import subprocess
    from shyft_amd.supervise import _free_port
    port = _free_port()
    deadline = time.monotonic() + float(os.environ.get("SHYFT_LAUNCH_DEADLINE_S", "3600"))
    procs = []
    for r in range(n_gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_gpus), LOCAL_WORLD_SIZE=str(n_gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)   # rank 0's supervisor hosts the store
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if live and time.monotonic() > deadline:
            print("bench.py: launcher wall deadline reached, ending the ranks", file=sys.stderr, flush=True)
            for q in live:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    return rc


def _progress(name):
    from shyft_amd.supervise import progress
    progress(name)


def dist_setup(n_gpus, use_gpu=True):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}: the line would not measure "
                         f"{n_gpus} GPU(s)")
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # GPU ranks: RCCL for device tensors, gloo for host tensors in the same group -- the host path the combines
        # fall back to if the RCCL self-check below fails (distributed.verify_collectives)
        backend = os.environ.get("SHYFT_DIST_BACKEND", "cpu:gloo,cuda:nccl" if use_gpu else "gloo")
        if use_gpu:
            # one rank per GPU (RCCL over xGMI). SHYFT_DIST_BACKEND=gloo + more ranks than GPUs is only for
            # rehearsing the multi-rank path on a one-GPU box; the device index wraps in that case.
            n_dev = torch.cuda.device_count()
            if "nccl" in backend and n_dev < world:
                raise SystemExit(f"bench.py: {world} ranks need {world} GPUs for RCCL, {n_dev} visible "
                                 f"(SHYFT_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
            local = local % n_dev if n_dev else local
            torch.cuda.set_device(local)
        from datetime import timedelta
        # a deadline on the rendezvous and on every collective (gloo raises, RCCL's watchdog aborts), below the
        # supervisor's stall limit, so that a stalled exchange ends this attempt rather than the whole run
        timeout = timedelta(seconds=float(os.environ.get("SHYFT_DIST_TIMEOUT_S", "180")))
        try:
            dist.init_process_group(backend, timeout=timeout)
        except Exception:  # noqa: BLE001 -- a torch without mixed-backend groups: RCCL alone (no host fallback)
            if backend != "cpu:gloo,cuda:nccl":
                raise
            dist.init_process_group("nccl", timeout=timeout)
        assert dist.get_world_size() == n_gpus
        _progress("rendezvous")
        pg = dist
        stall = os.environ.get("SHYFT_DIST_TEST_STALL", "")   # "rank:attempt": that rank stalls in the self-check
        if stall and stall == f"{rank}:{os.environ.get('SHYFT_SUPERVISE_ATTEMPT', '0')}":
            time.sleep(3600)   # (tests/test_bench_launch.py: the supervisor must replace this attempt)
        # one known-value all-gather, bit-exact on every rank, before any data uses the combines' path
        from shyft_amd import distributed
        nccl = "nccl" in str(dist.get_backend())
        if use_gpu:
            import torch
            distributed.verify_collectives(device=torch.device("cuda", local) if nccl else None)
        else:
            distributed.verify_collectives()
        _progress("self-check")
    return world, rank, local, pg


def _backend_name(pg):
    if pg is None:
        return "single rank"
    from shyft_amd import distributed
    b = str(pg.get_backend())
    name = "RCCL" if "nccl" in b and not distributed._COMBINE["host"] else "gloo (host)" if "gloo" in b else b
    return f"{name}; {distributed.combine_report()}"


def barrier_sync(pg, local, devices=None):
    import torch
    if pg is not None:
        pg.barrier()
    for d in sorted(set(devices)) if devices else [local]:
        torch.cuda.synchronize(d)


def max_over_ranks(pg, local, v: float) -> float:
    if pg is None:
        return v
    import torch
    from shyft_amd import distributed
    return distributed.max_over_ranks(v, device=torch.device("cuda", local))


def stack_defaults(stack, cells):
    from shyft_amd import synthetic
    if stack == "hbv_stack":
        return synthetic.default_hbv_parameters(), synthetic.default_hbv_state(cells)
    if stack == "pt_ss_k":
        return synthetic.default_ptssk_parameters(), synthetic.default_ptssk_state(cells)
    if stack == "pt_hs_k":
        return synthetic.default_pthsk_parameters(), synthetic.default_pthsk_state(cells)
    if stack == "pt_hps_k":
        return synthetic.default_pthpsk_parameters(), synthetic.default_pthpsk_state(cells)
    return synthetic.default_ptgsk_parameters(), synthetic.default_ptgsk_state(cells)


class Layout:
    """This rank's cells of the synthetic region: [off, off + n) of `total` cells, `n_catch` catchments in all.
    Weak scaling (default): every rank owns --cells cells, 100 catchments per shard. Strong scaling
    (--total-cells): the region is split by distributed.shard_range."""

    def __init__(self, a, world, rank, engine_gpus=0):
        from shyft_amd import distributed
        if engine_gpus:
            # the engine path: this process owns the whole region (its shards spread it over the GPUs)
            per = a.cells or (1 << 19 if a.stack == "hbv_stack" else 1 << 20)
            self.total = a.total_cells or per * engine_gpus
            self.off, self.n = 0, self.total
            self.n_catch = a.catchments or (100 if a.total_cells else 100 * engine_gpus)
            self.scaling = "strong" if a.total_cells else "weak"
            return
        if a.total_cells:
            b, e = distributed.shard_range(a.total_cells, world, rank)
            self.off, self.n, self.total = b, e - b, a.total_cells
            self.n_catch = a.catchments or 100
            self.scaling = "strong"
        else:
            self.n = a.cells or (1 << 19 if a.stack == "hbv_stack" else 1 << 20)
            self.off, self.total = rank * self.n, world * self.n
            self.n_catch = a.catchments or 100 * world
            self.scaling = "weak"


def build_region(stack, L, local, chunk, n_steps_axis, devices=None, shard_flags=0):
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K, HBV_STACK, PT_SS_K, PT_HS_K, PT_HPS_K, COLLECT_DISCHARGE
    sid = {"pt_gs_k": PT_GS_K, "hbv_stack": HBV_STACK, "pt_ss_k": PT_SS_K, "pt_hs_k": PT_HS_K, "pt_hps_k": PT_HPS_K}[stack]
    r = (HipRegion(sid, L.n, device=local) if devices is None else
         HipRegion(sid, L.n, devices=devices, shard_flags=shard_flags))
    r.set_geo(synthetic.geo11(L.n, n_catchments=L.n_catch, cell_offset=L.off, n_total=L.total))
    r.set_parameters(stack_defaults(stack, 1)[0])
    r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, n_steps_axis, chunk)
    r.set_collection(COLLECT_DISCHARGE)
    return r


class Router:
    """configs[4] routing (core/routing.h:239-421) over the synthetic river network of the whole region:
    per chunk each rank reduces its cells' avg_discharge to the global (river, UHG) group sums on its GPU and
    the partials are all-gathered and added in rank order (RCCL over xGMI); after the last chunk every rank
    convolves the network on its device (shyft_hip_route)."""

    def __init__(self, r, L, local, n_axis, pg):
        import torch
        from shyft_amd import api, synthetic
        self.n_catch = L.n_catch
        _, _, group = synthetic.cell_routing(L.n, self.n_catch, cell_offset=L.off, n_total=L.total)
        self.G = self.n_catch * len(synthetic.ROUTE_DISTANCES)
        r.set_routing_groups(group, self.G)
        self.group = group
        self.rivers = synthetic.river_network(self.n_catch)
        steps = [int((d / 1.0) / 3600.0 + 0.5) for d in synthetic.ROUTE_DISTANCES]
        self.group_uhgs = [api.make_uhg_from_gamma(steps[k], 7.0, 0.0) for _ in range(self.n_catch)
                           for k in range(len(steps))]
        self.group_river = [g // len(steps) for g in range(self.G)]
        self.river_uhgs = [api.make_uhg_from_gamma(int((d / v) / 3600.0 + 0.5), a, b) for (_, _, d, v, a, b) in self.rivers]
        self.river_down = [ds - 1 for (_, ds, *_rest) in self.rivers]
        self.dev = torch.device("cuda", local)
        self.sums = torch.zeros((self.G, n_axis), dtype=torch.float64, device=self.dev)
        self.part = None
        self.pg = pg
        self.out = None

    def attach(self, r):
        r.set_routing_groups(self.group, self.G)

    def chunk(self, r, step0, n):
        import torch
        from shyft_amd import distributed
        if self.part is None or self.part.shape[1] != n:
            self.part = torch.empty((self.G, n), dtype=torch.float64, device=self.dev)
        torch.cuda.synchronize(self.dev)
        r.routing_group_sums_device(step0, n, self.part.data_ptr())
        self.sums[:, step0:step0 + n] = distributed.combine_partials(self.part)

    def finish(self, T):
        import torch
        from shyft_amd.region import route
        s = self.sums[:, :T].contiguous()
        torch.cuda.synchronize(self.dev)
        self.out = route(None, self.group_uhgs, self.group_river, self.river_uhgs, self.river_down,
                         device=self.dev.index, sums_dev_ptr=s.data_ptr(), T=T)
        return self.out


class CatchmentSums:
    """Per-chunk catchment discharge sums of the whole region (cell_statistics::sum_catchment_feature over
    avg_discharge, core/cell_model.h:308-333; region_model::catchment_discharges, core/region_model.h:873-885):
    each rank reduces its cells per catchment on its GPU (shyft_hip_catchment_sums, deterministic segment
    sums), places the rows at their global catchment positions, and the partials are all-gathered (RCCL over
    xGMI) and added in rank order (distributed.combine_partials) into [C][T] on every rank."""

    def __init__(self, r, L, local, n_axis):
        import torch
        self.dev = torch.device("cuda", local)
        self.C = L.n_catch
        local_cids = [int(c) for c in r.catchment_ids()]
        self.rows = torch.tensor([c - 1 for c in local_cids], dtype=torch.long, device=self.dev)  # cid = 1 + index
        self.sums = torch.zeros((self.C, n_axis), dtype=torch.float64, device=self.dev)
        self.part = None
        self.full = None

    def chunk(self, r, step0, n):
        import torch
        from shyft_amd import distributed
        if self.part is None or self.part.shape[1] != n:
            self.part = torch.empty((len(self.rows), n), dtype=torch.float64, device=self.dev)
            self.full = torch.zeros((self.C, n), dtype=torch.float64, device=self.dev)
        r.catchment_sums_device(0, step0, n, self.part.data_ptr())   # synchronous on the region's stream
        self.full.index_copy_(0, self.rows, self.part)
        distributed.combine_partials(self.full, out=self.sums[:, step0:step0 + n])


def run_year(r, L, chunk, k_steps, seed, stations=None, router=None, btk=False, btk_ms=None,
             r_alt=None, sums=None, walls=None, parts=None, overlap=0, idw_ms=None):
    """K bench steps from Jan 1: per chunk put the chunk's forcing into HBM (device generator,
    or IDW / BTK from the station network), then run_cells (and the routing group sums).

    With r_alt (a second region over the same cells) and the device generator, the chunks alternate between
    the two regions: chunk s+1's forcing is generated into the other region's window on its own stream while
    chunk s runs, and the state is handed over device to device (shyft_hip_copy_state) before chunk s+1 runs.
    Every chunk's forcing is still produced inside the timed region; the generator just no longer adds to it."""
    if r_alt is not None and stations is None:
        return _run_year_pipelined((r, r_alt), L, chunk, k_steps, seed, router, sums)
    if overlap and stations is None:
        return _run_year_overlapped(r, L, chunk, k_steps, seed, router, sums, walls, parts, overlap)
    kernel_ms = []
    for s in range(k_steps):
        _progress(f"chunk {s}")
        t_chunk = time.perf_counter()
        step0 = s * chunk
        # the chunk's forcing rows are all rewritten below and run_cells writes every response row of the
        # window, so the window moves without the NaN pre-fill of set_window
        r.move_window(step0, 0)
        if stations is None:
            r.synthetic_forcing(seed, step0, chunk, cell_offset=L.off)
        else:
            xyz, vals = stations
            v = vals[s % len(vals)]
            gms = [0.0] * 5
            for var in range(5):
                if var == 0 and btk:
                    t = time.perf_counter()
                    r.interpolate_btk(xyz, v[0], step0, BTK_DEFAULTS)   # synchronous
                    if btk_ms is not None:
                        btk_ms.append((time.perf_counter() - t) * 1e3)
                else:
                    r.interpolate(var, xyz, v[var], step0, IDW_DEFAULTS[var])
                    gms[var] = r.last_interpolate_ms()   # the gather kernel alone (HIP events)
            if idw_ms is not None:
                idw_ms.append(gms)
        r.run_cells(0, step0, chunk)
        kernel_ms.append(r.last_run_ms())
        if parts is not None:
            parts.append(r.last_run_kernel_ms())
        if sums is not None:
            sums.chunk(r, step0, chunk)
        if router is not None:
            router.chunk(r, step0, chunk)
        if walls is not None:
            _sync()
            walls.append((time.perf_counter() - t_chunk) * 1e3)
    if router is not None:
        router.finish(k_steps * chunk)
    return kernel_ms


def _sync():
    import torch
    torch.cuda.synchronize()


def _run_year_overlapped(r, L, chunk, k_steps, seed, router, sums, walls, parts, n_cus):
    """As run_year with the device generator, but chunk s+1's forcing is generated into the region's second window
    buffer on a side stream while chunk s runs (shyft_hip_prefetch_synthetic_forcing), and the buffers swap before
    chunk s+1 (the run waits for the generator on the device). n_cus > 0: the side stream is restricted to that many
    CUs; n_cus < 0: the whole device at the lowest stream priority, enqueued after chunk s's run, so the run's
    workgroups are dispatched first and the generator's fill the CUs its tail leaves idle. Chunk 0's forcing is
    generated before its run, inside the timed region like every other chunk's."""
    kernel_ms = []
    r.move_window(0, 0)
    r.synthetic_forcing(seed, 0, chunk, cell_offset=L.off)
    for s in range(k_steps):
        _progress(f"chunk {s}")
        t_chunk = time.perf_counter()
        step0 = s * chunk
        if n_cus < 0:
            r.run_cells_async(step0, chunk)
            if s + 1 < k_steps:
                r.prefetch_synthetic_forcing(seed, step0 + chunk, cell_offset=L.off, n_cus=n_cus)
            r.synchronize()   # the run's error check (region_model::run_cells semantics)
        else:
            if s + 1 < k_steps:
                r.prefetch_synthetic_forcing(seed, step0 + chunk, cell_offset=L.off, n_cus=n_cus)
            r.run_cells(0, step0, chunk)
        kernel_ms.append(r.last_run_ms())
        if parts is not None:
            parts.append(r.last_run_kernel_ms())
        if sums is not None:
            sums.chunk(r, step0, chunk)
        if router is not None:
            router.chunk(r, step0, chunk)
        if s + 1 < k_steps:
            r.swap_forcing_window(step0 + chunk)
        if walls is not None:
            _sync()
            walls.append((time.perf_counter() - t_chunk) * 1e3)
    if router is not None:
        router.finish(k_steps * chunk)
    return kernel_ms


def _run_year_pipelined(regs, L, chunk, k_steps, seed, router, sums):
    kernel_ms = []
    regs[0].move_window(0, 0)
    regs[0].synthetic_forcing(seed, 0, chunk, cell_offset=L.off)
    for s in range(k_steps):
        cur, nxt = regs[s % 2], regs[(s + 1) % 2]
        step0 = s * chunk
        cur.run_cells_async(step0, chunk)
        if s + 1 < k_steps:
            # host-synchronous on nxt's stream only: the generator overlaps cur's kernel
            nxt.move_window(step0 + chunk, 0)
            nxt.synthetic_forcing(seed, step0 + chunk, chunk, cell_offset=L.off)
        cur.synchronize()   # error check of the run (region_model::run_cells semantics)
        kernel_ms.append(cur.last_run_ms())
        if s + 1 < k_steps:
            nxt.copy_state_from(cur)
        if sums is not None:
            sums.chunk(cur, step0, chunk)
        if router is not None:
            router.chunk(cur, step0, chunk)
    if router is not None:
        router.finish(k_steps * chunk)
    return kernel_ms


def cpu_baseline(stack, n_cells, threads):
    """Reference-scheduler CPU run (oracle built with host libm) on n_cells x 8760."""
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K
    from tests import oracle_lib
    run = {"hbv_stack": oracle_lib.hbv_run, "pt_ss_k": oracle_lib.ptssk_run, "pt_hs_k": oracle_lib.pthsk_run,
           "pt_hps_k": oracle_lib.pthpsk_run}.get(stack, oracle_lib.ptgsk_run)
    # forcing of the sample cells: identical bits from the device generator (tests/test_capi.py pins equality)
    g = HipRegion(PT_GS_K, n_cells, device=0)
    g.set_geo(synthetic.geo11(n_cells, n_total=1 << 20))
    g.set_parameters(synthetic.default_ptgsk_parameters())
    g.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, YEAR)
    g.synthetic_forcing(synthetic.SEED, 0, YEAR)
    f = np.stack([g.get_forcing(v, 0, YEAR) for v in range(5)])
    g.close()
    geo = synthetic.geo11(n_cells, n_total=1 << 20)
    p, st = stack_defaults(stack, n_cells)
    res = run(geo, p, st, synthetic.T0_2015_US, synthetic.HOUR_US, f, ncore=threads, variant="libm")
    el = res["elapsed_s"]
    # single-core rate on a small slice
    n1 = min(200, n_cells)
    r1 = run(geo[:n1], p, st[:n1], synthetic.T0_2015_US, synthetic.HOUR_US, np.ascontiguousarray(f[:, :, :n1]),
             ncore=1, variant="libm")
    return {
        "value": n_cells * YEAR / el,
        "unit": "cell-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_cells} cells x {YEAR} hourly steps of the same synthetic region (first cells of the 1M-cell "
                  f"region), oracle restatement built with host libm, reference scheduler "
                  f"(region_model.h:991-1021) with use_ncore={threads}; run_cells wall {el:.2f}s",
        "single_core_value": n1 * YEAR / r1["elapsed_s"],
        "cpu_model": _cpu_model(),
    }


def cpu_baseline_idw(n_cells, threads):
    """configs[2] on the CPU: the oracle's inverse-distance interpolation (oracle/src/idw.hpp, restating
    core/inverse_distance.h:142-250; host libm) of the five variables from the same 500-station network onto the first
    n_cells cells of the 1M-cell region, then the pt_gs_k oracle with the reference scheduler, over the year."""
    from shyft_amd import synthetic
    from tests import oracle_lib
    xyz = station_network(1 << 20)
    vals = station_values(xyz, 0, YEAR)                      # [5][YEAR][S], prepared before timing (an input)
    geo = synthetic.geo11(n_cells, n_total=1 << 20)
    dst = np.ascontiguousarray(geo[:, 0:3])
    kinds = (0, 1, 3, 4, 2)                                  # oracle kinds of T, P, WS, RH, RAD
    t0 = time.perf_counter()
    f = np.stack([oracle_lib.idw_run(kinds[v], xyz, vals[v], dst, IDW_DEFAULTS[v],
                                     dst_slope=geo[:, 5] if v == 4 else None, variant="libm") for v in range(5)])
    t_idw = time.perf_counter() - t0
    p, st = stack_defaults("pt_gs_k", n_cells)
    res = oracle_lib.ptgsk_run(geo, p, st, synthetic.T0_2015_US, synthetic.HOUR_US, f, ncore=threads, variant="libm")
    el = t_idw + res["elapsed_s"]
    return {
        "value": n_cells * YEAR / el,
        "unit": "cell-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_cells} cells x {YEAR} hourly steps of the configs[2] region (first cells of the 1M-cell region, "
                  f"{N_STATIONS} stations): oracle IDW of the 5 variables (host libm, destinations split over up to 16 "
                  f"threads: {t_idw:.2f} s) + pt_gs_k oracle with the reference scheduler, use_ncore={threads} "
                  f"({res['elapsed_s']:.2f} s)",
        "idw_s": t_idw,
        "run_cells_s": res["elapsed_s"],
        "cpu_model": _cpu_model(),
    }


PROFILE_DIR = os.path.join(ROOT, "profiles", "r06")


def workload_tag(a, cells):
    """Key of a workload for the committed PMC summaries: they are only used for the exact same run."""
    return (f"{a.stack}{'_idw' if a.idw else ''}{'_btk' if a.btk else ''}_c{cells}_k{a.chunk}"
            f"_s{a.steps}_w{a.warmup}{f'_sh{a.shards}' if a.shards > 1 else ''}")


def pmc_summary(a, cells, suffix=""):
    """(summary, reason): the committed rocprofv3 PMC summary of the dominant kernel
    (profiles/<round>/pmc_<workload>.json, written by tools/gpu_profile.sh + tools/pmc_summary.py from this same
    bench command) -- only if it measured THIS build of the library (same sha256), else (None, why). PMC counters
    cannot be read from inside this process."""
    from shyft_amd import _native
    rel = f"profiles/{os.path.basename(PROFILE_DIR)}/pmc_{workload_tag(a, cells)}{suffix}.json"
    try:
        d = json.load(open(os.path.join(ROOT, rel)))
    except (OSError, ValueError):
        return None, f"no PMC summary of this workload ({rel})"
    sha = _native.lib_sha()
    if d.get("lib_sha256") != sha:
        return None, (f"{rel} measured library sha256 {str(d.get('lib_sha256'))[:16]}, this run loads "
                      f"{sha[:16]}: counters of another build are not reported")
    return d, None


SEASONS = (("winter (Dec-Feb)", (12, 1, 2)), ("spring (Mar-May)", (3, 4, 5)), ("summer (Jun-Aug)", (6, 7, 8)),
           ("autumn (Sep-Nov)", (9, 10, 11)))


def _chunk_month(step0, n):
    """calendar month (1-12) of the middle of steps [step0, step0 + n) of the synthetic year (2015, hourly)"""
    import datetime
    mid = datetime.datetime(2015, 1, 1) + datetime.timedelta(hours=(step0 + n / 2.0) % YEAR)
    return mid.month


def instruction_budget(a, pmc, timed, cells, chunk):
    """the run kernel's VALU lane-instructions per cell-step by season (SQ_INSTS_VALU of each
    timed launch of the PMC pass), by instruction class (the SQ_INSTS_VALU_* pass), and -- pt_gs_k -- next to the CPU
    oracle's fp64 operation count for the same steps (tools/mb/ptgsk_opcount.cpp: every add / mul / div / fma of the
    restatement counted as it runs, on 1024 cells of the same region)."""
    per = 64.0 / (cells * chunk)
    months = [_chunk_month(k * chunk, chunk) for k in range(len(timed))]
    by_season = {}
    for name, ms in SEASONS:
        v = [l["SQ_INSTS_VALU"] * per for l, m in zip(timed, months) if m in ms]
        if v:
            by_season[name] = round(float(np.mean(v)), 1)
    out = {"lane_instr_per_cell_step_by_season": by_season}
    if "valu_lane_instr_per_cell_step_by_class" in pmc:
        out["lane_instr_per_cell_step_by_class"] = {k: round(v, 1) for k, v in
                                                   pmc["valu_lane_instr_per_cell_step_by_class"].items()}
    if a.stack == "pt_gs_k" and not a.idw and chunk == CHUNK:
        try:
            oc = json.load(open(os.path.join(PROFILE_DIR, "ptgsk_oracle_opcount_1024cells.json")))
        except (OSError, ValueError):
            return out
        rows = oc["per_cell_step_by_chunk"]
        ops = {}
        for name, ms in SEASONS:
            v = [r["add"] + r["mul"] + r["div"] + r["fma"] + r["sqrt"] for k, r in enumerate(rows)
                 if _chunk_month(k * chunk, chunk) in ms]
            d = [r["div"] for k, r in enumerate(rows) if _chunk_month(k * chunk, chunk) in ms]
            if v:
                ops[name] = {"fp64_ops": round(float(np.mean(v)), 1), "of_which_divisions": round(float(np.mean(d)), 1)}
        out["oracle_fp64_ops_per_cell_step_by_season"] = ops
        out["oracle_fp64_ops_source"] = (f"profiles/{os.path.basename(PROFILE_DIR)}/ptgsk_oracle_opcount_1024cells.json "
                                         "(tools/mb/ptgsk_opcount.cpp: the oracle with a counting double type, 1024 "
                                         "cells of the bench region, the same 438-step chunks); a division is one "
                                         "operation there and about ten VALU instructions on gfx950")
    return out


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def dist_check(a, world, rank, pg):
    """--dist-check: the bench's launcher, rendezvous and catchment-sum combination without HIP. Each rank
    sums a synthetic per-cell series (the generator's temperature of its shard) per catchment, the partials
    go through distributed.combine_partials in rank order, and rank 0 compares with the unsharded sums."""
    import torch
    from shyft_amd import distributed, synthetic
    L = Layout(a, world, rank)
    T = 48
    def sums_of(off, n):
        cid = synthetic.geo11(n, n_catchments=L.n_catch, cell_offset=off, n_total=L.total)[:, 4].astype(np.int64)
        f = synthetic.forcing(n, 0, T, synthetic.SEED, cell_offset=off)[0]            # [T][n]
        out = np.zeros((L.n_catch, T))
        for c in np.unique(cid):
            out[c - 1] = f[:, cid == c].sum(axis=1)
        return out
    total = distributed.combine_partials(torch.from_numpy(sums_of(L.off, L.n))).numpy()
    wall = distributed.max_over_ranks(float(rank + 1))
    if rank == 0:
        ref = sums_of(0, L.total)
        print(json.dumps({"dist_check": True, "n_gpus": world, "backend": pg.get_backend() if pg else None,
                          "cells": L.total, "catchments": L.n_catch, "max_over_ranks": wall,
                          "max_abs_diff": float(np.abs(total - ref).max()),
                          "checksum": float(total.sum()), "combine": distributed.combine_report(),
                          "supervisor": supervisor_info()}), flush=True)
    if pg is not None:
        pg.destroy_process_group()


def supervisor_info():
    """The `supervisor` field of a rank's line: which attempt produced it and why the one before ended."""
    if os.environ.get("SHYFT_SUPERVISED") != "1":
        return None
    return {"attempt": int(os.environ.get("SHYFT_SUPERVISE_ATTEMPT", "0")),
            "combines": os.environ.get("SHYFT_SUPERVISE_MODE", ""),
            "previous_attempt": os.environ.get("SHYFT_SUPERVISE_REASON", "") or None,
            "note": "each rank process supervises its rank as a child and restarts all ranks with gloo combines if "
                    "the RCCL attempt fails or stalls (shyft_amd/supervise.py)"}


def main():
    a = parse()
    if a.launch is None:
        a.launch = "ranks" if a.gpus > 1 else "engine"
    engine = "WORLD_SIZE" not in os.environ and a.launch == "engine" and not a.dist_check
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not engine:
        sys.exit(launch_ranks(a.gpus))
    if "WORLD_SIZE" in os.environ and not engine and int(os.environ["WORLD_SIZE"]) != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: the line would not "
                         f"measure {a.gpus} GPU(s)")
    if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and os.environ.get("SHYFT_SUPERVISED") != "1"
            and os.environ.get("SHYFT_NO_SUPERVISE") != "1"):
        # a rank process (torch.distributed.run's or launch_ranks'): supervise the real rank as a child. Nothing here
        # has touched the GPU.
        from shyft_amd.supervise import supervise
        sys.exit(supervise([sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    _progress("start")
    devices = None
    if engine and (a.gpus > 1 or a.shards > 1):
        # one process, the region's cells in shards over the GPUs (the engine's multi-GPU path)
        devices = [k % a.gpus for k in range(a.shards or a.gpus)]
    world, rank, local, pg = dist_setup(1 if devices else a.gpus, use_gpu=not a.dist_check)
    if a.dist_check:
        return dist_check(a, world, rank, pg)
    import torch  # noqa: F401  (device init / sync)
    from shyft_amd import synthetic

    n_dev = len(set(devices)) if devices else world
    L = Layout(a, world, rank, engine_gpus=n_dev if devices else 0)
    cells = L.total // n_dev if devices else L.n      # per GPU (the shards of one GPU run concurrently)
    if a.overlap_forcing is None:
        # a region of at most 2 workgroups per CU leaves the GPU under-filled: its next window's forcing is generated
        # beside the run at the lowest stream priority (measured r06, 131,072 cells: 7.21e9 -> 7.38e9 cell-steps/s);
        # a full region generates before its run (overlapping it slowed the 1M-cell run kernel 42.1 -> 48.1 ms,
        # profiles/r06/forcing_overlap_variants.txt)
        a.overlap_forcing = -1 if (cells <= SMALL_REGION_CELLS and not a.idw and not a.btk and not a.pipeline) else 0
    chunk = a.chunk
    n_axis = max(YEAR, (max(a.steps, a.warmup)) * chunk)
    from shyft_amd.region import SHARD_BALANCE_Z
    r = build_region(a.stack, L, local, chunk, n_axis, devices, SHARD_BALANCE_Z if a.balance_z else 0)
    _progress("region")
    state0 = stack_defaults(a.stack, L.n)[1]
    read_b, write_b, state_b, kernel_name = STACKS[a.stack]
    stations = None
    if a.btk:
        a.idw = True
    if a.idw:
        # station series prepared on the host before timing (the reference's region_env input);
        # each step uploads its chunk (14.6 MB) and interpolates 5 variables on the GPU
        xyz = station_network(L.total)
        stations = (xyz, [station_values(xyz, s * chunk, chunk) for s in range(max(a.steps, a.warmup))])

    routing = (a.routing or a.stack == "pt_ss_k") and not a.no_routing
    router = Router(r, L, local, n_axis, pg) if routing else None
    sums = None if a.no_catchment_sums else CatchmentSums(r, L, local, n_axis)
    r_alt = None
    if not a.idw and a.pipeline:
        r_alt = build_region(a.stack, L, local, chunk, n_axis)
        if router is not None:
            router.attach(r_alt)

    # warmup (untimed): W chunks from Jan 1, then state is reset for the timed year
    if a.warmup > 0:
        r.set_state(state0)
        run_year(r, L, chunk, a.warmup, synthetic.SEED, stations, router, a.btk, r_alt=r_alt, sums=sums,
                 overlap=a.overlap_forcing)
    r.set_state(state0)   # the initial state is an input: resident in HBM before the timed region
    barrier_sync(pg, local, devices)
    t0 = time.perf_counter()
    btk_ms = []
    walls, parts = [], []
    idw_ms = []
    kernel_ms = run_year(r, L, chunk, a.steps, synthetic.SEED, stations, router, a.btk, btk_ms,
                         r_alt=r_alt, sums=sums, walls=walls, parts=parts, overlap=a.overlap_forcing, idw_ms=idw_ms)
    barrier_sync(pg, local, devices)
    wall = time.perf_counter() - t0
    wall = max_over_ranks(pg, local, wall)
    avg_kernel_ms = max_over_ranks(pg, local, float(np.mean(kernel_ms)))
    # per-chunk wall (max over ranks) and the calendar year: the timed chunks 1-12 are Jan..Dec of one year
    walls = [max_over_ranks(pg, local, w) for w in walls] if walls else []

    total_cell_steps = L.total * chunk * a.steps
    value = total_cell_steps / wall
    bytes_per_launch = cells * chunk * (read_b + write_b) + cells * state_b
    # engine shards sharing a device run concurrently, each timed by its own events: no single launch spans the
    # device's kernel time, so the bytes of all its shards are priced over the step's wall time (a lower bound)
    shared = bool(devices) and len(devices) > len(set(devices))
    roof_ms = wall * 1e3 / a.steps if shared else avg_kernel_ms
    achieved = bytes_per_launch / (roof_ms * 1e-3)
    pmc, pmc_missing = pmc_summary(a, cells)
    traffic_b = None if pmc is None else pmc["traffic_bytes_per_launch"]
    out = {
        "metric": METRIC if a.stack == "pt_gs_k" else METRIC.replace("pt_gs_k", a.stack),
        "value": value,
        "unit": "cell-steps/s",
        "n_gpus": n_dev,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": L.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8d generator, seed 20251015; " +
                ("500 stations, BTK temperature + IDW per chunk)" if a.btk else
                 "500 stations, IDW per chunk)" if a.idw else "device-generated per chunk)"),
        "config": {
            "workload": (f"{a.stack} + bayesian kriging temperature + inverse_distance from {N_STATIONS} stations, "
                         if a.btk else f"{a.stack} + inverse_distance from {N_STATIONS} stations, " if a.idw
                         else f"{a.stack} ") +
                        f"region_model::run_cells, {cells} cells/GPU x {chunk * a.steps} hourly steps "
                        f"({a.steps} chunks of {chunk}), discharge_collector, default "
                        f"{dict(hbv_stack='HbvParameter', pt_ss_k='PTSSKParameter', pt_hs_k='PTHSKParameter', pt_hps_k='PTHPSKParameter').get(a.stack, 'PTGSKParameter')}",
            "cells_per_gpu": cells,
            "total_cells": L.total,
            "catchments": L.n_catch,
            "steps_per_chunk": chunk,
            "forcing": ("IDW/BTK from stations, per chunk, before its run" if a.idw else
                        ("device generator, chunk s+1 into a second window buffer on a whole-device lowest-priority "
                         "side stream enqueued after chunk s's run (chunk 1 before its run); every chunk's forcing is "
                         "generated inside the timed region" if a.overlap_forcing < 0 else
                         f"device generator, chunk s+1 into a second window buffer on a {a.overlap_forcing}-CU side "
                         "stream while chunk s runs (chunk 1 before its run)") if a.overlap_forcing else
                        "device generator, per chunk, overlapped with the previous chunk's run (two regions, state "
                        "handed over device to device)" if r_alt is not None else
                        "device generator, per chunk, before its run"),
            "parallelism": (f"one process, the region in {len(devices)} engine shards over {n_dev} GPU(s) "
                            f"(shyft_hip_region_create_sharded), no data-path collective"
                            + ("" if sums is None else "; per-chunk catchment discharge sums all-gathered inside "
                               f"the engine ({r.combine_path().upper()}) and added in shard order")
                            + f"; combine: {r.combine_report()}"
                            if devices else
                            f"cells sharded over {world} GPU(s), one process each, no data-path collective"
                            + ("" if sums is None else "; per-chunk catchment discharge sums all-gathered "
                               f"({_backend_name(pg)}) and added in rank order")),
        },
        "kernel_ms_per_step": avg_kernel_ms,
        "kernel_cell_steps_per_s": L.total * chunk / (avg_kernel_ms * 1e-3),
        "chunk_wall_ms": [round(w, 2) for w in walls],
        **({"shard_kernel_ms_last_chunk": [round(x, 2) for x in r.shard_run_ms()]} if devices else {}),
        "chunk_kernel_ms": [round(k, 2) for k in kernel_ms],
        "roofline": {
            "bound": "hbm",
            "achieved": achieved / 1e9,
            "peak": HBM_PEAK_BPS / 1e9,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_BPS,
            "traffic": None if traffic_b is None else traffic_b / (roof_ms * 1e-3) / 1e9,
            "time_basis": ("step wall time: the device's shards run concurrently" if shared else
                           "mean kernel launch time (HIP events on the region's stream)"),
            "traffic_bytes_per_launch": traffic_b,
            "traffic_source": (pmc_missing if pmc is None else
                               f"profiles/{os.path.basename(PROFILE_DIR)}/pmc_{workload_tag(a, cells)}.json "
                               f"(library sha256 {pmc['lib_sha256'][:16]}, the one this run loaded): rocprofv3 "
                               f"FETCH_SIZE x {pmc['calibration']['fetch_correction']:.3f} + WRITE_SIZE x "
                               f"{pmc['calibration']['write_correction']:.3f} (gfx950 correction calibrated in the same "
                               "run, tools/pmc_summary.py), mean over the timed launches of this same command, over "
                               "this run's mean launch duration"),
            "kernel": kernel_name,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "note": f"{read_b + write_b} B/cell-step ({read_b} B forcing read + {write_b} B discharge/charge write) + "
                    f"{state_b} B/cell state per launch (DESIGN.md)",
        },
    }
    if len(walls) >= YEAR // chunk and chunk * (YEAR // chunk) == YEAR:
        ny = YEAR // chunk
        out["calendar_year"] = {
            "value": L.total * chunk * ny / (sum(walls[:ny]) * 1e-3), "unit": "cell-steps/s",
            "chunks": f"timed chunks 1-{ny} (Jan 1 - Dec 31, {YEAR} hourly steps: " + {
                "pt_gs_k": "BASELINE configs[2]'s year" if a.idw else "BASELINE configs[1]'s year",
                "hbv_stack": "BASELINE configs[3]'s year", "pt_ss_k": "the first year of BASELINE configs[4]'s 3-year "
                "horizon"}.get(a.stack, "one calendar year") + ")",
            "ms_per_step": sum(walls[:ny]) / ny,
            "kernel_ms_per_step": float(np.mean(kernel_ms[:ny])),
            "note": "per-chunk wall clocks of this same timed run (synchronised at the end of each chunk)"}
    if a.btk:
        # the BTK time loop per chunk: one fp64 GEMM [cells x (S+3)] x [(S+3) x chunk], plus host
        # work (source rows, per-step beta); the full-set operators are built on the first chunk and reused
        ms = max_over_ranks(pg, local, float(np.mean(btk_ms)))
        flops = 2.0 * cells * (N_STATIONS + 3) * chunk
        out["btk"] = {
            "ms_per_chunk": ms,
            "cell_steps_per_s": L.total * chunk / (ms * 1e-3),
            "roofline": {"bound": "fp64", "achieved": flops / (ms * 1e-3) / 1e12, "peak": FP64_PEAK_FLOPS / 1e12,
                         "unit": "TFLOP/s", "frac": flops / (ms * 1e-3) / FP64_PEAK_FLOPS,
                         "write_GBps": cells * chunk * 8 / (ms * 1e-3) / 1e9,
                         "note": "2 * cells * (stations + 3) * chunk flops per call over its wall time "
                                 "(host part included)"},
        }
    if a.idw and not a.btk and idw_ms:
        # configs[2]'s interpolation: the five IDW gathers of every chunk (kernels/idw.hip), HBM-bound accounting as
        # the run kernel's, over the gathers' own HIP-event times
        per_var = [float(max_over_ranks(pg, local, float(np.mean([c[v] for c in idw_ms])))) for v in range(5)]
        b_var = [idw_gather_bytes(v, cells, chunk) for v in range(5)]
        ms_chunk = float(sum(per_var))
        ipmc, ipmc_missing = pmc_summary(a, cells, suffix="_idw_gather")
        itraffic = None if ipmc is None else ipmc["traffic_bytes_per_launch_sum"]
        out["idw"] = {
            "kernel_ms_per_chunk": ms_chunk,
            "share_of_chunk_wall": ms_chunk / (wall * 1e3 / a.steps),
            "by_variable_ms": dict(zip(("temperature", "precipitation", "wind_speed", "rel_hum", "radiation"),
                                       [round(x, 3) for x in per_var])),
            "roofline": {
                "bound": "hbm", "achieved": sum(b_var) / (ms_chunk * 1e-3) / 1e9, "peak": HBM_PEAK_BPS / 1e9,
                "unit": "GB/s", "frac": sum(b_var) / (ms_chunk * 1e-3) / HBM_PEAK_BPS,
                "temperature_GBps": b_var[0] / (per_var[0] * 1e-3) / 1e9,
                "traffic": None if itraffic is None else itraffic / (ms_chunk * 1e-3) / 1e9,
                "traffic_bytes_per_chunk": itraffic,
                "traffic_source": ipmc_missing if ipmc is None else
                f"profiles/{os.path.basename(PROFILE_DIR)}/pmc_{workload_tag(a, cells)}_idw_gather.json (library "
                f"sha256 {ipmc['lib_sha256'][:16]}, the one this run loaded): the five gathers' FETCH_SIZE x "
                f"{ipmc['calibration']['fetch_correction']:.3f} + WRITE_SIZE per chunk, mean over the timed chunks",
                "valu_busy": None if ipmc is None else ipmc["valu_busy"],
                "algorithmic_bytes_per_chunk": sum(b_var),
                "kernel": "idw_wave_gather_kernel (5 launches per chunk, one per forcing variable)",
                "note": "algorithmic bytes: 8 B written per cell-step + the neighbour tables and source rows read "
                        "once per launch (bench.idw_gather_bytes)"},
        }
    if pmc is not None:
        # the bound that does apply to the VALU-bound stacks: fp64 VALU issue. SQ_ACTIVE_INST_VALU (quad-cycles of
        # VALU issue summed over waves) per timed launch of the same command, over this run's mean kernel time on
        # 1024 SIMDs at 2.4 GHz
        timed = pmc["launches"][pmc["warmup"]:]
        act = float(np.mean([l["SQ_ACTIVE_INST_VALU"] for l in timed]))
        ins = float(np.mean([l["SQ_INSTS_VALU"] for l in timed]))
        out["valu"] = {
            "busy": act * 4.0 / (1024 * 2.4e9 * avg_kernel_ms * 1e-3),
            "wave_instr_per_launch": ins,
            "lane_instr_per_cell_step": ins * 64.0 / (cells * chunk),
            **instruction_budget(a, pmc, timed, cells, chunk),
            "by_chunk_busy": [round(l["valu_busy"], 3) for l in timed],
            "profile_kernel_ms": pmc["trace_mean_ms_timed"],
            "source": f"profiles/{os.path.basename(PROFILE_DIR)}/pmc_{workload_tag(a, cells)}.json (rocprofv3 SQ "
                      "pass of this same command); busy = SQ_ACTIVE_INST_VALU*4 / (1024 SIMDs x 2.4 GHz x this "
                      "run's mean kernel time); by_chunk_busy uses each PMC launch's own duration; "
                      "profile_kernel_ms = the --kernel-trace pass's mean over the timed launches",
        }
    if router is not None:
        o = router.out[2]
        out["config"]["workload"] += (f"; routing::uhg through a {len(router.rivers)}-river network "
                                      f"({router.G} (river, UHG) groups all-gathered per chunk, network convolved on "
                                      f"device after the last chunk)")
        out["routing"] = {"rivers": len(router.rivers), "groups": router.G,
                          "outlet_mean_m3s": float(o[0].mean()), "outlet_max_m3s": float(o[0].max())}
        if a.dump_route and rank == 0:
            np.save(a.dump_route, np.stack(router.out))
    if sums is not None:
        T = a.steps * chunk
        tot = sums.sums[:, :T]
        out["catchment_sums"] = {"catchments": sums.C, "series": "avg_discharge", "steps": T,
                                 "checksum": float(tot.sum().item()),
                                 "note": "per chunk: segment sums on each GPU, allgather + rank-order add (inside "
                                         "the timed region)"}
        if a.dump_sums and rank == 0:
            np.save(a.dump_sums, tot.cpu().numpy())
    if supervisor_info() is not None:
        out["supervisor"] = supervisor_info()
    if rank == 0 and world == 1 and not devices and not a.no_cpu_baseline:
        threads = a.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        out["cpu_baseline"] = (cpu_baseline_idw(a.cpu_cells, threads) if a.idw and not a.btk and a.stack == "pt_gs_k"
                               else cpu_baseline(a.stack, a.cpu_cells, threads))
    if rank == 0:
        print(json.dumps(out), flush=True)
    r.close()
    if r_alt is not None:
        r_alt.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
