"""Kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage (CPU, no GPU needed).
usage: python tools/kres.py <file.hip> <name-regex> [extra hipcc flags...]"""
import re
import subprocess
import sys

src, pat, flags = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3:]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                      "-Wno-unused-function", *flags, "-c", src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, cwd="shyft_amd/csrc")
cur = None
rows = {}
for line in out.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]):\s*(\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k.split(" [")[0]] = v
for name, r in rows.items():
    if pat.search(name):
        short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)[:60]
        print(f"{short:60s} vgpr {r.get('VGPRs','?'):>4} spill {r.get('VGPRs Spill','?'):>4} sspill {r.get('SGPRs Spill','?'):>4} "
              f"scratch {r.get('ScratchSize','?'):>4} occ {r.get('Occupancy','?')} lds {r.get('LDS Size','?')}")
if out.returncode:
    print(out.stderr[-2000:])
