"""Read tools/mb/probe_hwid's dump: per wavefront HW_ID, XCC_ID, start / end s_memtime (see probe_hwid.hip).

Reports: the SIMD of each wave index within its workgroup, the TG_ID values, and -- for every pair of workgroups
that overlap in time on the same CU -- whether their solver wavefronts (device/wave_place.h: the wave on SIMD
TG_ID & 3, else wave 0) sit on different SIMDs, against the old choice (wave 0)."""
import collections
import sys

import numpy as np

a = np.fromfile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/probe_hwid.bin", dtype=np.uint32).reshape(-1, 4, 6)
hw = a[:, :, 0]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
tg = (hw >> 16) & 15
xcc = a[:, :, 1] & 15
t0 = a[:, 0, 2].astype(np.uint64) | (a[:, 0, 3].astype(np.uint64) << np.uint64(32))
t1 = a[:, 0, 4].astype(np.uint64) | (a[:, 0, 5].astype(np.uint64) << np.uint64(32))
nb = a.shape[0]
print(f"{nb} workgroups; distinct SIMDs within a workgroup: {collections.Counter(len(set(simd[b])) for b in range(nb))}")
print("SIMD of wave 0:", collections.Counter(simd[:, 0].tolist()))
print("TG_ID:", sorted(collections.Counter(tg[:, 0].tolist()).items()))
print("waves of one workgroup on one CU:", all(len(set(zip(xcc[b], se[b], sh[b], cu[b]))) == 1 for b in range(nb)))


def solver(b, placed):
    if placed:
        for w in range(4):
            if simd[b, w] == (tg[b, 0] & 3):
                return int(simd[b, w])
    return int(simd[b, 0])


key = [(int(xcc[b, 0]), int(se[b, 0]), int(sh[b, 0]), int(cu[b, 0])) for b in range(nb)]
by_cu = collections.defaultdict(list)
for b in range(nb):
    by_cu[key[b]].append(b)
print(f"CUs seen: {len(by_cu)}; workgroups per CU: {collections.Counter(len(v) for v in by_cu.values())}")
for placed in (False, True):
    same = diff = 0
    load = collections.Counter()
    for bs in by_cu.values():
        for i in range(len(bs)):
            for j in range(i + 1, len(bs)):
                p, q = bs[i], bs[j]
                if t0[p] < t1[q] and t0[q] < t1[p]:
                    if solver(p, placed) == solver(q, placed):
                        same += 1
                    else:
                        diff += 1
        # the most solvers on one SIMD among workgroups overlapping the CU's first workgroup
        b0 = bs[0]
        ov = [b for b in bs if t0[b] < t1[b0] and t0[b0] < t1[b]]
        load[max(collections.Counter(solver(b, placed) for b in ov).values())] += 1
    print(f"{'TG_ID-placed' if placed else 'wave 0'} solver: overlapping pairs on the same SIMD {same}, "
          f"on different SIMDs {diff}; max solvers per SIMD among the first workgroup's co-residents: {dict(load)}")
