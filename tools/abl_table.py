"""Per-chunk SQ counters of tools/r03_ablate.sh runs: VALU lane-instructions per cell-step per variant."""
import csv
import sys
from collections import defaultdict

CS = (1 << 20) * 730


def load(path, kernel="ptgsk_run_kernel"):
    d = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


if __name__ == "__main__":
    names = sys.argv[1:]
    rows = {n: load(f"gpurun_out/pmc_abl_{n}/p1/run_counter_collection.csv") for n in names}
    print("chunk " + " ".join(f"{n:>12}" for n in names))
    for c in range(12):
        print(f"{c:5d} " + " ".join(f"{rows[n][c]['SQ_INSTS_VALU'] * 64 / CS:12.0f}" for n in names))
    print("mean  " + " ".join(f"{sum(r['SQ_INSTS_VALU'] for r in rows[n]) * 64 / CS / 12:12.0f}" for n in names))
    print("SALU  " + " ".join(f"{sum(r['SQ_INSTS_SALU'] for r in rows[n]) * 64 / CS / 12:12.0f}" for n in names))
