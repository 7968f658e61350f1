"""Print inputs where the device's v_max3/min3 (ops 11/12) or chained v_max (op 13) differ from numpy fmax/fmin chains."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import forma_rt as fr
from test_gpu_parity import _edge_floats

rng = np.random.default_rng(12)
fp = C.POINTER(C.c_float)
x = _edge_floats(rng, 50000)
y = np.roll(_edge_floats(rng, 50000), 3)[: x.size]
z = np.roll(y, -1)
out = np.empty_like(x)
for op, f in ((11, np.fmax), (12, np.fmin), (13, np.fmax)):
    fr.check(fr.lib().fr_selftest_ops(0, op, x.ctypes.data_as(fp), y.ctypes.data_as(fp), x.size, out.ctypes.data_as(fp)))
    want = f(f(x, y), z)
    bad = ~((np.isnan(out) & np.isnan(want)) | (out.view(np.uint32) == want.view(np.uint32)))
    idx = np.nonzero(bad)[0]
    print(f"op {op}: {idx.size} mismatches")
    for i in idx[:12]:
        print("  ", [hex(int(v)) for v in (x[i:i+1].view(np.uint32)[0], y[i:i+1].view(np.uint32)[0], z[i:i+1].view(np.uint32)[0])],
              x[i], y[i], z[i], "got", out[i], hex(int(out[i:i+1].view(np.uint32)[0])), "want", want[i])
