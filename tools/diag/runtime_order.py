"""Which HIP runtime copies get mapped, and whether the engine and torch can both initialise,
for the two import/initialisation orders.  usage: python tools/diag/runtime_order.py A|B"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

order = sys.argv[1]
if order == "A":          # engine library first
    from oversim_amd import kbr
    kbr.lib()
    import torch
else:                     # torch first
    import torch
    from oversim_amd import kbr
    kbr.lib()
maps = open("/proc/self/maps").read()
print(order, "runtimes:", sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "hsa-runtime" in l)))
from oversim_amd import KbrEngine
if order == "A":
    e = KbrEngine(0); print("engine ok")
    print("torch", torch.cuda.is_available(), torch.zeros(4, device="cuda").sum().item())
else:
    print("torch", torch.cuda.is_available(), torch.zeros(4, device="cuda").sum().item())
    e = KbrEngine(0); print("engine ok")
