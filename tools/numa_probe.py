import os, glob, json
out = {"affinity": sorted(os.sched_getaffinity(0))[:64], "n_affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node*")):
    try:
        nodes[os.path.basename(d)] = open(d + "/cpulist").read().strip()
    except OSError:
        pass
out["nodes"] = nodes
import sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from ray_memory_management_amd._native import require_hip
h = require_hip()
bus = h.pci_bus_id(0)
out["pci_bus_id"] = bus
cands = glob.glob("/sys/bus/pci/devices/*")
m = [c for c in cands if c.lower().endswith(str(bus).lower()) or str(bus).lower() in c.lower()]
out["match"] = m[:3]
for c in m[:1]:
    try:
        out["gpu_numa_node"] = open(c + "/numa_node").read().strip()
        out["local_cpulist"] = open(c + "/local_cpulist").read().strip()
    except OSError as e:
        out["err"] = repr(e)
print(json.dumps(out))
