"""Summarise the rocprofv3 passes of tools/gpu_profile.sh (gpurun_out/prof_{trace,fetch,write,sq}) for one bench
command into profiles/<round>/pmc_<workload>.json -- the file bench.py reads for that same command's `traffic`
and `valu` fields.

Launches of the dominant kernel are matched by dispatch order across the passes (each pass is a fresh run of the
same command); the first `warmup` launches are the bench's untimed warmup chunks and are reported apart. Over the
timed launches:
  fetch / write bytes: FETCH_SIZE and WRITE_SIZE (KiB -> bytes). MI355X_MICROARCH.md ("HBM [CDNA4]"): on gfx950
      FETCH_SIZE reports half the bytes of a wide coalesced streaming read, WRITE_SIZE reads exactly. The kernels
      here load and store 8 B per lane, a width the guide does not calibrate, so the same run calibrates it with
      two kernels of known byte counts: the forcing generator writes exactly 40 B per cell-step (5 fp64 rows) and
      the catchment segment sums read the 8 B discharge of every cell-step once. fetch_correction = algorithmic
      read bytes / FETCH bytes of the segment sums (the guide's factor 2 when it holds), applied to the kernel's
      FETCH; write_correction likewise from the generator.
  traffic = fetch * fetch_correction + write * write_correction per launch
  valu_busy = SQ_ACTIVE_INST_VALU * 4 / (1024 SIMDs * duration * 2.4 GHz) (quad-cycles of VALU issue; a lower
      bound if the clock runs below its 2.4 GHz maximum)
  trace_mean_ms: the kernel's mean duration in the --kernel-trace --stats pass (timed launches; all launches too)
usage: python tools/pmc_summary.py [--kernel K] [--round r02] [--bench-args "..."] [--base gpurun_out]
"""
import argparse
import csv
import json
import os
import shlex
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SIMDS = 256 * 4
CLOCK = 2.4e9


def counter_rows(path, kname):
    rows = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        if kname not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = {"duration_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "grid": int(r["Grid_Size"]),
                   "scratch_bytes_per_lane": int(r["Scratch_Size"]), "vgpr": int(r["VGPR_Count"])}
    return [(d, rows[d], meta[d]) for d in sorted(rows)]


def trace_durations(path, kname):
    out = []
    for r in csv.DictReader(open(path)):
        if kname in r["Kernel_Name"]:
            out.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    return [ms for _, ms in sorted(out)]


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="ptgsk_run_kernel")
    ap.add_argument("--round", default="r06")
    ap.add_argument("--bench-args", default="--gpus 1 --steps 20 --warmup 5")
    ap.add_argument("--base", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--idw", action="store_true",
                    help="summarise the five IDW gathers of each chunk (idw_wave_gather_kernel) of a --idw command into "
                         "pmc_<workload>_idw_gather.json instead of the run kernel")
    o = ap.parse_args()
    if o.idw:
        return idw_main(o)
    import bench
    a = bench.parse(shlex.split(o.bench_args))
    L = bench.Layout(a, 1, 0)
    cells, chunk, W = L.n, a.chunk, a.warmup
    read_b, write_b, state_b, _ = bench.STACKS[a.stack]

    f = counter_rows(os.path.join(o.base, "prof_fetch", "run_counter_collection.csv"), o.kernel)
    w = counter_rows(os.path.join(o.base, "prof_write", "run_counter_collection.csv"), o.kernel)
    q = counter_rows(os.path.join(o.base, "prof_sq", "run_counter_collection.csv"), o.kernel)
    if not f or len(f) != len(w) or len(f) != len(q):
        raise SystemExit(f"launch counts differ across passes: {len(f)} {len(w)} {len(q)}")
    # calibration kernels (same runs)
    gen_w = counter_rows(os.path.join(o.base, "prof_write", "run_counter_collection.csv"), "synthetic_forcing_kernel")
    seg_f = counter_rows(os.path.join(o.base, "prof_fetch", "run_counter_collection.csv"), "segment_sum_kernel")
    gen_bytes = cells * chunk * 40.0
    seg_bytes = cells * chunk * 8.0
    # the region's generator launches (not cpu_baseline's 4000-cell sample; --idw runs have none)
    gen_w = [g for g in gen_w if g[2]["grid"] >= cells]
    write_ratio = mean([r["WRITE_SIZE"] * 1024.0 / gen_bytes for _, r, m in gen_w]) if gen_w else None
    # the catchment sums (one workgroup per step and catchment, contiguous cell blocks, so coalesced rows);
    # routing group sums use the same kernel on hash-scattered cells (gathers) and are not a calibration
    seg_grid = chunk * L.n_catch * 256
    seg_ratios = [r["FETCH_SIZE"] * 1024.0 / seg_bytes for _, r, m in seg_f if m["grid"] == seg_grid]
    fetch_ratio = mean(seg_ratios) if seg_ratios else None
    fetch_corr = 1.0 / fetch_ratio if fetch_ratio else 2.0
    write_corr = 1.0 / write_ratio if write_ratio else 1.0

    # optional pass 5: VALU instructions by class (tools/gpu_profile.sh "sqf")
    qf_path = os.path.join(o.base, "prof_sqf", "run_counter_collection.csv")
    qf = counter_rows(qf_path, o.kernel) if os.path.exists(qf_path) else []
    if qf and len(qf) != len(f):
        raise SystemExit(f"VALU-class pass launch count {len(qf)} != {len(f)}")
    launches = []
    for n_l, ((df, cf, mf), (dw, cw, mw), (dq, cq, mq)) in enumerate(zip(f, w, q)):
        fb = cf["FETCH_SIZE"] * 1024.0
        wb = cw["WRITE_SIZE"] * 1024.0
        dur = mq["duration_ns"] * 1e-9
        launches.append({"dispatch": [df, dw, dq], "fetch_bytes": fb, "write_bytes": wb,
                         "traffic_bytes": fb * fetch_corr + wb * write_corr,
                         "sq_duration_ns": mq["duration_ns"],
                         "valu_busy": cq["SQ_ACTIVE_INST_VALU"] * 4.0 / (SIMDS * dur * CLOCK), **cq, **mq,
                         **({("class_" + k): v for k, v in qf[n_l][1].items()} if qf else {})})
    timed = launches[W:]
    tr = trace_durations(os.path.join(o.base, "prof_trace", "run_kernel_trace.csv"), o.kernel)
    algo = cells * chunk * (read_b + write_b) + cells * state_b
    lib_sha = _sha(o.base)
    res = {
        "lib_sha256": lib_sha,
        "command": f"python3 bench.py {o.bench_args} under rocprofv3 (tools/gpu_profile.sh: one --kernel-trace "
                   f"--stats pass, then one --pmc pass per counter group, each a fresh run of the same command)",
        "workload": bench.workload_tag(a, cells),
        "kernel": o.kernel, "cells": cells, "chunk": chunk, "steps": a.steps, "warmup": W,
        "calibration": {
            "write_ratio_generator": write_ratio,
            "fetch_ratio_segment_sum": fetch_ratio,
            "fetch_correction": fetch_corr, "write_correction": write_corr,
            "note": "ratio = counter bytes / known bytes of the same run's forcing generator (40 B/cell-step "
                    "written) and catchment segment sums (8 B/cell-step read); corrections are 1/ratio",
        },
        "algorithmic_bytes_per_launch": algo,
        "fetch_bytes_per_launch": mean([l["fetch_bytes"] for l in timed]),
        "write_bytes_per_launch": mean([l["write_bytes"] for l in timed]),
        "traffic_bytes_per_launch": mean([l["traffic_bytes"] for l in timed]),
        "valu_busy": mean([l["valu_busy"] for l in timed]),
        "valu_wave_instr_per_launch": mean([l["SQ_INSTS_VALU"] for l in timed]),
        "trace_mean_ms_timed": mean(tr[W:]),
        "trace_mean_ms_all": mean(tr),
        "trace_launches": len(tr),
        "launches": launches,
    }
    res["traffic_over_algorithmic"] = res["traffic_bytes_per_launch"] / algo
    if qf:
        # lane-instructions per cell-step by class, mean over the timed launches (wave instructions x 64 lanes)
        per = 64.0 / (cells * chunk)
        cls = {"fp64_add": "SQ_INSTS_VALU_ADD_F64", "fp64_mul": "SQ_INSTS_VALU_MUL_F64",
               "fp64_fma": "SQ_INSTS_VALU_FMA_F64", "fp64_trans": "SQ_INSTS_VALU_TRANS_F64",
               "int32": "SQ_INSTS_VALU_INT32", "int64": "SQ_INSTS_VALU_INT64", "cvt": "SQ_INSTS_VALU_CVT"}
        res["valu_lane_instr_per_cell_step_by_class"] = {
            k: mean([l["class_" + c] for l in timed]) * per for k, c in cls.items()}
        res["valu_lane_instr_per_cell_step_by_class"]["all"] = mean([l["class_SQ_INSTS_VALU"] for l in timed]) * per
    out_dir = os.path.join(ROOT, "profiles", o.round)
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"pmc_{res['workload']}.json")
    json.dump(res, open(out, "w"), indent=1)
    import shutil
    stats = os.path.join(o.base, "prof_trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out_dir, f"stats_{res['workload']}.csv"))
    print(out)
    print(json.dumps({k: res[k] for k in ("traffic_bytes_per_launch", "traffic_over_algorithmic", "valu_busy",
                                          "trace_mean_ms_timed", "trace_mean_ms_all", "calibration")}))


def _sha(base):
    sha_path = os.path.join(base, "lib_sha.txt")
    if not os.path.exists(sha_path):
        raise SystemExit(f"{sha_path} missing: the passes must record the sha256 of the library they measured "
                         "(tools/gpu_profile.sh)")
    return open(sha_path).read().strip()


def idw_main(o):
    """configs[2]'s interpolation: per chunk the five gathers (one per forcing variable, in forcing order), summed."""
    import bench
    a = bench.parse(shlex.split(o.bench_args))
    L = bench.Layout(a, 1, 0)
    cells, chunk, W = L.n, a.chunk, a.warmup
    kname = "idw_wave_gather_kernel"
    f = counter_rows(os.path.join(o.base, "prof_fetch", "run_counter_collection.csv"), kname)
    w = counter_rows(os.path.join(o.base, "prof_write", "run_counter_collection.csv"), kname)
    q = counter_rows(os.path.join(o.base, "prof_sq", "run_counter_collection.csv"), kname)
    if not f or len(f) != len(w) or len(f) != len(q) or len(f) % 5:
        raise SystemExit(f"gather launch counts differ across passes or are not 5 per chunk: {len(f)} {len(w)} {len(q)}")
    seg_f = counter_rows(os.path.join(o.base, "prof_fetch", "run_counter_collection.csv"), "segment_sum_kernel")
    seg_grid = chunk * L.n_catch * 256
    seg_ratios = [r["FETCH_SIZE"] * 1024.0 / (cells * chunk * 8.0) for _, r, m in seg_f if m["grid"] == seg_grid]
    fetch_corr = 1.0 / mean(seg_ratios) if seg_ratios else 2.0
    algo = [bench.idw_gather_bytes(v, cells, chunk) for v in range(5)]
    chunks = []
    for c in range(len(f) // 5):
        fb = [f[5 * c + v][1]["FETCH_SIZE"] * 1024.0 for v in range(5)]
        wb = [w[5 * c + v][1]["WRITE_SIZE"] * 1024.0 for v in range(5)]
        dur = [q[5 * c + v][2]["duration_ns"] * 1e-9 for v in range(5)]
        act = [q[5 * c + v][1]["SQ_ACTIVE_INST_VALU"] for v in range(5)]
        chunks.append({"fetch_bytes": fb, "write_bytes": wb,
                       "traffic_bytes": [x * fetch_corr + y for x, y in zip(fb, wb)],
                       "duration_ms": [d * 1e3 for d in dur],
                       "valu_busy": [x * 4.0 / (SIMDS * d * CLOCK) for x, d in zip(act, dur)]})
    timed = chunks[W:]
    tr = trace_durations(os.path.join(o.base, "prof_trace", "run_kernel_trace.csv"), kname)
    tr_chunks = [sum(tr[5 * c:5 * c + 5]) for c in range(len(tr) // 5)]
    res = {
        "lib_sha256": _sha(o.base),
        "command": f"python3 bench.py {o.bench_args} under rocprofv3 (tools/gpu_profile.sh passes)",
        "workload": bench.workload_tag(a, cells), "kernel": kname, "cells": cells, "chunk": chunk, "warmup": W,
        "calibration": {"fetch_correction": fetch_corr, "write_correction": 1.0,
                        "note": "FETCH correction from the same run's catchment segment sums (8 B/cell-step read); "
                                "WRITE_SIZE as counted (the guide: exact on gfx950)"},
        "algorithmic_bytes_by_variable": algo,
        "traffic_bytes_by_variable": [mean([c["traffic_bytes"][v] for c in timed]) for v in range(5)],
        "traffic_bytes_per_launch_sum": mean([sum(c["traffic_bytes"]) for c in timed]),
        "valu_busy_by_variable": [mean([c["valu_busy"][v] for c in timed]) for v in range(5)],
        "valu_busy": mean([sum(b * d for b, d in zip(c["valu_busy"], c["duration_ms"])) / sum(c["duration_ms"])
                           for c in timed]),
        "trace_mean_ms_by_variable": [mean(tr[5 * W + v::5]) for v in range(5)],
        "trace_mean_ms_chunk_timed": mean(tr_chunks[W:]),
        "chunks": chunks,
    }
    res["traffic_over_algorithmic"] = res["traffic_bytes_per_launch_sum"] / sum(algo)
    out_dir = os.path.join(ROOT, "profiles", o.round)
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"pmc_{res['workload']}_idw_gather.json")
    json.dump(res, open(out, "w"), indent=1)
    print(out)
    print(json.dumps({k: res[k] for k in ("traffic_over_algorithmic", "valu_busy", "valu_busy_by_variable",
                                          "trace_mean_ms_by_variable", "trace_mean_ms_chunk_timed")}))


if __name__ == "__main__":
    main()
