import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
order = sys.argv[1]
def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})
if order == "torch_first":
    import torch
    print("torch cuda", torch.cuda.is_available(), torch.cuda.device_count())
from shyft_amd.region import HipRegion, PT_GS_K
r = HipRegion(PT_GS_K, 10)
print("maps after region", maps())
import torch
print("torch available", torch.cuda.is_available())
x = torch.zeros(3, device="cuda:0"); print("torch ok", x.sum().item())
print("maps end", maps())
