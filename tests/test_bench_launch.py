"""bench.py's multi-rank path (BASELINE configs[3]/[4] at N>1).

`bench.py --gpus N --launch ranks` without an outside launcher starts N rank processes itself (a parent that never
touches the GPU), every rank asserts WORLD_SIZE == N, and the per-chunk catchment discharge sums are all-gathered and
added in rank order (distributed.combine_partials). CPU tests drive that launcher, rendezvous and collective
with gloo (--dist-check); the GPU tests run the real sharded HipRegion bench with two ranks on one GPU
(SHYFT_DIST_BACKEND=gloo) and compare the combined catchment sums with a single-rank run of the same region.

The default N > 1 path without a launcher is the engine's (--launch engine): one process, the region in one shard
per GPU (shyft_hip_region_create_sharded), the partial sums combined inside the engine. On a one-GPU box
`--gpus 1 --shards K` runs K shards on device 0 through the same code (device-copy combination).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("world,cells,catch", [(2, 10001, 37), (3, 4096, 100)])
def test_launcher_gloo_dist_check(world, cells, catch):
    p, out = _bench(["--gpus", str(world), "--dist-check", "--total-cells", str(cells), "--catchments", str(catch)])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["n_gpus"] == world and out["backend"] == "gloo"
    assert out["max_over_ranks"] == float(world)
    # rank-order sums of shard partials vs the unsharded sums (catchments split across ranks reassociate)
    assert out["max_abs_diff"] < 1e-9


@pytest.mark.parametrize("stalled", [1, 0])
def test_stalled_self_check_restarts_ranks_with_host_combines(stalled):
    """One rank stalls inside the collective self-check of the first attempt (SHYFT_DIST_TEST_STALL): its supervisor
    sees no progress within the stall limit, every rank's child is killed and replaced by a fresh one (no process that
    ran is re-executed), and the second attempt -- gloo combines -- prints the line, saying why the first ended."""
    t0 = __import__("time").monotonic()
    p, out = _bench(["--gpus", "2", "--dist-check", "--total-cells", "4096"],
                    env_extra={"SHYFT_DIST_TEST_STALL": f"{stalled}:0", "SHYFT_SUPERVISE_STALL_S": "6",
                               "SHYFT_SUPERVISE_FIRST_S": "120", "SHYFT_DIST_TIMEOUT_S": "60"}, timeout=240)
    took = __import__("time").monotonic() - t0
    assert p.returncode == 0, p.stderr[-3000:]
    assert out is not None and out["max_abs_diff"] < 1e-9
    sup = out["supervisor"]
    assert sup["attempt"] == 1 and sup["combines"] == "gloo"
    assert "made no progress" in sup["previous_attempt"] or "exited with status" in sup["previous_attempt"]
    assert took < 120, took   # the stall limit (6 s) and two start-ups, far below the collective timeout (60 s)
    assert len([l for l in p.stdout.splitlines() if l.startswith("{")]) == 1


def test_first_attempt_line_carries_supervisor_field():
    p, out = _bench(["--gpus", "2", "--dist-check", "--total-cells", "4096"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["supervisor"]["attempt"] == 0 and out["supervisor"]["previous_attempt"] is None


def _torchrun(world, args, env_extra=None, timeout=300):
    """The driver's N > 1 command: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
    127.0.0.1 --master-port P bench.py --gpus N ... (torchrun's agent hosts the store the supervisors share)."""
    from shyft_amd.supervise import _free_port
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world)] + args
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


def test_torchrun_gloo_dist_check():
    p, out = _torchrun(2, ["--dist-check", "--total-cells", "4096"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["n_gpus"] == 2 and out["max_abs_diff"] < 1e-9 and out["supervisor"]["attempt"] == 0
    assert len([l for l in p.stdout.splitlines() if l.startswith("{")]) == 1


def test_torchrun_stalled_self_check_restarts_ranks_with_host_combines():
    """The same stall as above under torch.distributed.run: the supervisors agree over torchrun's agent store."""
    p, out = _torchrun(2, ["--dist-check", "--total-cells", "4096"],
                       env_extra={"SHYFT_DIST_TEST_STALL": "1:0", "SHYFT_SUPERVISE_STALL_S": "6",
                                  "SHYFT_SUPERVISE_FIRST_S": "120", "SHYFT_DIST_TIMEOUT_S": "60"}, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    assert out is not None and out["max_abs_diff"] < 1e-9
    assert out["supervisor"]["attempt"] == 1 and out["supervisor"]["combines"] == "gloo"


def test_world_size_mismatch_fails():
    p, out = _bench(["--gpus", "2", "--dist-check"], env_extra={"WORLD_SIZE": "3", "RANK": "0"})
    assert p.returncode != 0 and out is None
    assert "WORLD_SIZE=3" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("stack", ["pt_gs_k", "hbv_stack"])
def test_two_ranks_one_gpu_catchment_sums_match_single_rank(stack, tmp_path):
    """Two real ranks (gloo on one GPU) over a 4096-cell region == one rank over the same region: the shard
    boundary (cell 2048) falls on a catchment boundary, so every catchment is summed by one rank and the
    rank-order combination adds zeros; the sums must agree bit for bit."""
    common = ["--stack", stack, "--total-cells", "4096", "--catchments", "100", "--chunk", "48", "--steps", "3",
              "--warmup", "0", "--no-cpu-baseline", "--no-routing"]
    p1, o1 = _bench(["--gpus", "1", "--dump-sums", str(tmp_path / "s1.npy")] + common)
    assert p1.returncode == 0, p1.stderr[-2000:]
    p2, o2 = _bench(["--gpus", "2", "--launch", "ranks", "--dump-sums", str(tmp_path / "s2.npy")] + common,
                    env_extra={"SHYFT_DIST_BACKEND": "gloo"})
    assert p2.returncode == 0, p2.stderr[-2000:]
    assert o1["n_gpus"] == 1 and o2["n_gpus"] == 2 and o2["scaling"] == "strong"
    s1, s2 = np.load(tmp_path / "s1.npy"), np.load(tmp_path / "s2.npy")
    assert s1.shape == (100, 144) and np.isfinite(s1).all() and s1.sum() > 0
    assert np.array_equal(s1, s2)


@pytest.mark.gpu
def test_torchrun_two_ranks_one_gpu_match_single_rank(tmp_path):
    """The driver's launcher (torch.distributed.run) over the real GPU bench: two supervised ranks on one device
    (gloo combines: RCCL cannot hold two ranks of one communicator on one device) give the single rank's sums."""
    common = ["--total-cells", "4096", "--catchments", "100", "--chunk", "48", "--steps", "3", "--warmup", "0",
              "--no-cpu-baseline"]
    p1, o1 = _bench(["--gpus", "1", "--dump-sums", str(tmp_path / "s1.npy")] + common)
    assert p1.returncode == 0, p1.stderr[-2000:]
    p2, o2 = _torchrun(2, ["--dump-sums", str(tmp_path / "s2.npy")] + common, env_extra={"SHYFT_DIST_BACKEND": "gloo"})
    assert p2.returncode == 0, p2.stderr[-2000:]
    assert o2["n_gpus"] == 2 and o2["supervisor"]["attempt"] == 0
    assert np.array_equal(np.load(tmp_path / "s1.npy"), np.load(tmp_path / "s2.npy"))


@pytest.mark.gpu
@pytest.mark.parametrize("world,cells", [(2, 4096), (3, 4099)])
def test_sharded_routing_matches_single_rank(world, cells, tmp_path):
    """configs[4]'s routing (core/routing.h:344-383) through the real multi-rank bench path: every rank forms the
    (river, UHG) group sums of its own cells, the partials are all-gathered and added in rank order, then every rank
    convolves the river network. Two ranks split 4096 cells on a catchment boundary, so each group is summed on
    one rank and the result must equal one rank's bit for bit; three ranks over 4099 cells split groups between
    ranks, so the group sums reassociate: the routed series then agree within 1e-12 of their magnitude."""
    common = ["--stack", "pt_ss_k", "--total-cells", str(cells), "--catchments", "100", "--chunk", "48", "--steps",
              "3", "--warmup", "0", "--no-cpu-baseline", "--no-catchment-sums"]
    p1, o1 = _bench(["--gpus", "1", "--dump-route", str(tmp_path / "r1.npy")] + common)
    assert p1.returncode == 0, p1.stderr[-2000:]
    pn, on = _bench(["--gpus", str(world), "--launch", "ranks", "--dump-route", str(tmp_path / "rn.npy")] + common,
                    env_extra={"SHYFT_DIST_BACKEND": "gloo"})
    assert pn.returncode == 0, pn.stderr[-2000:]
    assert o1["n_gpus"] == 1 and on["n_gpus"] == world and "routing" in on
    r1, rn = np.load(tmp_path / "r1.npy"), np.load(tmp_path / "rn.npy")
    assert r1.shape[0] == 3 and r1.shape[2] == 144 and np.isfinite(r1).all() and r1[2].sum() > 0
    if world == 2:
        assert np.array_equal(r1, rn)
    else:
        scale = np.abs(r1).max()
        assert np.max(np.abs(r1 - rn)) <= 1e-12 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("cus", ["8", "-1"])
def test_overlapped_forcing_generation_same_results(tmp_path, cus):
    """bench --overlap-forcing (chunk s+1's forcing generated into a second window buffer on a side stream -- 8 CUs,
    or the whole device at the lowest priority enqueued after chunk s's run -- then swapped in) gives the same
    catchment sums as generating each chunk before its run: the same generator, the same rows, the run waits for the
    generator on the device and the generator for the run that last read its buffer."""
    common = ["--total-cells", "20000", "--catchments", "50", "--chunk", "96", "--steps", "4", "--warmup", "1",
              "--no-cpu-baseline"]
    p0, o0 = _bench(["--dump-sums", str(tmp_path / "a.npy")] + common)
    assert p0.returncode == 0, p0.stderr[-2000:]
    p1, o1 = _bench(["--dump-sums", str(tmp_path / "b.npy"), "--overlap-forcing", cus] + common)
    assert p1.returncode == 0, p1.stderr[-2000:]
    a, b = np.load(tmp_path / "a.npy"), np.load(tmp_path / "b.npy")
    assert a.shape == (50, 384) and np.isfinite(a).all() and a.sum() > 0
    assert np.array_equal(a, b)
    assert "second window buffer" in o1["config"]["forcing"]


@pytest.mark.gpu
@pytest.mark.parametrize("stack", ["pt_gs_k", "pt_ss_k"])
def test_engine_shards_one_process_match_unsharded(stack, tmp_path):
    """bench's single-process engine path with two shards on device 0: the per-chunk catchment discharge sums and
    (pt_ss_k) the routed river series equal the unsharded region's bit for bit (the shard boundary, cell 2048, is a
    catchment boundary; routing groups follow catchments)."""
    common = ["--stack", stack, "--total-cells", "4096", "--catchments", "100", "--chunk", "48", "--steps", "3",
              "--warmup", "0", "--no-cpu-baseline"]
    p1, o1 = _bench(["--gpus", "1", "--dump-sums", str(tmp_path / "s1.npy"), "--dump-route", str(tmp_path / "r1.npy")]
                    + common)
    assert p1.returncode == 0, p1.stderr[-2000:]
    p2, o2 = _bench(["--gpus", "1", "--shards", "2", "--dump-sums", str(tmp_path / "s2.npy"),
                     "--dump-route", str(tmp_path / "r2.npy")] + common)
    assert p2.returncode == 0, p2.stderr[-2000:]
    assert o2["n_gpus"] == 1 and "2 engine shards" in o2["config"]["parallelism"]
    assert "COPY" in o2["config"]["parallelism"]
    assert np.array_equal(np.load(tmp_path / "s1.npy"), np.load(tmp_path / "s2.npy"))
    if stack == "pt_ss_k":
        r1, r2 = np.load(tmp_path / "r1.npy"), np.load(tmp_path / "r2.npy")
        assert r1[2].sum() > 0 and np.array_equal(r1, r2)
