"""Summarise the rocprofv3 passes of tools/gpu_profile.sh (gpurun_out/prof_{trace,fetch,write,sq}) for the
bench's dominant kernel into profiles/<round>/<stack>_pmc.json, the file bench.py reads its `traffic` from.

Per launch of the kernel (matched by dispatch order across the separate PMC passes, each a fresh run of the
same bench command):
  traffic  = FETCH_SIZE + WRITE_SIZE (KiB as reported -> bytes; no gfx950 x2 correction: the kernel's loads are
             8 B/lane, a width MI355X_MICROARCH.md does not calibrate)
  valu_busy = SQ_ACTIVE_INST_VALU * 4 / (SIMDs * duration * clock): the fraction of SIMD cycles issuing VALU
             (SQ_ACTIVE_INST_* count quad-cycles; 1024 SIMDs; clock = 2.4 GHz, the MI355X maximum, so this is a
             lower bound when the clock runs below it)
  valu_instr_per_s = SQ_INSTS_VALU / duration (wave instructions)
usage: python tools/pmc_summary.py <kernel-name-substring> <cells> <chunk> <out.json> [gpurun_out]
"""
import csv
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
CLOCK = 2.4e9


def launches(path, kname):
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


def main():
    kname, cells, chunk, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    base = sys.argv[5] if len(sys.argv) > 5 else "gpurun_out"
    f = launches(os.path.join(base, "prof_fetch", "run_counter_collection.csv"), kname)
    w = launches(os.path.join(base, "prof_write", "run_counter_collection.csv"), kname)
    q = launches(os.path.join(base, "prof_sq", "run_counter_collection.csv"), kname)
    res = {"command": "tools/gpu_profile.sh: rocprofv3 --kernel-trace --pmc <counters> -- python3 bench.py "
                      "--no-cpu-baseline --steps 12 --warmup 0 (one pass per counter group; a full year of 730-step chunks)",
           "kernel": kname, "cells": cells, "chunk": chunk, "launches": []}
    fetch, write, busy, ips = [], [], [], []
    for (df, cf, mf), (dw, cw, mw), (dq, cq, mq) in zip(f, w, q):
        fb = cf["FETCH_SIZE"] * 1024.0
        wb = cw["WRITE_SIZE"] * 1024.0
        dur = mq["duration_ns"] * 1e-9
        vb = cq["SQ_ACTIVE_INST_VALU"] * 4.0 / (SIMDS * dur * CLOCK)
        fetch.append(fb)
        write.append(wb)
        busy.append(vb)
        ips.append(cq["SQ_INSTS_VALU"] / dur)
        res["launches"].append({"dispatch": [df, dw, dq], "fetch_bytes": fb, "write_bytes": wb,
                                "sq_duration_ns": mq["duration_ns"], "valu_busy": vb, **cq, **mq})
    n = len(fetch)
    if n == 0:
        raise SystemExit("no launches of " + kname)
    res["fetch_bytes_per_launch"] = sum(fetch) / n
    res["write_bytes_per_launch"] = sum(write) / n
    res["traffic_bytes_per_launch"] = (sum(fetch) + sum(write)) / n
    res["valu_busy"] = sum(busy) / n
    res["valu_wave_instr_per_s"] = sum(ips) / n
    res["algorithmic_bytes_per_launch"] = cells * chunk * 56 + cells * 144
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("traffic_bytes_per_launch", "valu_busy", "valu_wave_instr_per_s")}))


if __name__ == "__main__":
    main()
