import os, sys, tempfile, uuid
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from ray_memory_management_amd._native import require_hip, store_ext
h = require_hip()
name = "/rmm-dbg-" + uuid.uuid4().hex[:8]
host = store_ext().ObjectStore.create_segment(name, 512 << 20, tempfile.mkdtemp(), 0.8, 1 << 20, True)
g = h.GpuStore(0, 96 << 20, 32 << 20, name, True)
s = torch.cuda.current_stream().cuda_stream
xs, ids = [], []
for i in range(8):
    x = (torch.randn(8 << 20, device="cuda") * (i + 1)).to(torch.bfloat16)
    oid = os.urandom(20)
    g.put_segments(oid, [(x.data_ptr(), x.numel() * 2)], 16, s)
    xs.append(x); ids.append(oid)
    print("put", i, g.stats()["spilled_objects"], host.stats()["num_objects"], flush=True)
for i, (x, oid) in enumerate(zip(xs, ids)):
    try:
        t = torch.from_dlpack(h.store_dlpack(g, oid, [x.numel()], 4, 16, s))
    except Exception as e:
        print("GET FAILED", e, "| last transfer error:", g.last_error(), g.stats(), h.h2d_stats(), h.host_register_last_error())
        for o in host.list_objects():
            print({k: (v.hex() if isinstance(v, bytes) else v) for k, v in o.items()})
        raise
    ok = torch.equal(t, x)
    del t
    print("get", i, ok, g.stats()["spilled_objects"], g.stats()["restored_bytes_total"], host.stats()["num_objects"], flush=True)
print("last_error after gets:", g.last_error())
print("h2d stats", h.h2d_stats(), "reg error:", h.host_register_last_error())
for oid in ids:
    g.delete(oid)
print("after delete host objects:", host.stats()["num_objects"])
for o in host.list_objects():
    print({k: (v.hex() if isinstance(v, bytes) else v) for k, v in o.items()})
print("gpu stats", g.stats())
print("last error:", g.last_error())
