"""Which step of a bench process narrows its CPU affinity:
prints len(os.sched_getaffinity(0)) at start, after numpy, after torch, after the
HIP runtime's initialisation, and after libge's load."""
import json
import os
import sys

out = {"start": len(os.sched_getaffinity(0))}
import numpy  # noqa: E402,F401
out["numpy"] = len(os.sched_getaffinity(0))
import torch  # noqa: E402
out["torch_import"] = len(os.sched_getaffinity(0))
torch.cuda.init()
torch.zeros(1, device="cuda:0")
out["hip_init"] = len(os.sched_getaffinity(0))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-embed_amd", "py"))
import ge_amd  # noqa: E402
ge_amd.lib()
c = ge_amd.Context(0)
out["libge_context"] = len(os.sched_getaffinity(0))
c.close()
out["env"] = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OMP_PROC_BIND", "OMP_PLACES",
                                             "GOMP_CPU_AFFINITY", "HIP_VISIBLE_DEVICES")}
with open("/proc/self/status") as f:
    out["cpus_allowed_list"] = [l.split(":", 1)[1].strip() for l in f if l.startswith("Cpus_allowed_list")]
print(json.dumps(out))
