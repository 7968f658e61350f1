"""Print the exhaustive recip_nr mismatch table (per exponent field) on GPU 0."""
import ctypes as C
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "fo-rma_amd"))
import forma_rt as fr

bad = np.zeros(256, np.uint64)
first = np.zeros(256, np.uint32)
L = fr.lib()
rc = L.fr_selftest_recip(0, 0, 1 << 32, bad.ctypes.data_as(C.POINTER(C.c_uint64)), first.ctypes.data_as(C.POINTER(C.c_uint32)))
fr.check(rc)
print("total mismatches:", int(bad.sum()))
for e in range(256):
    if bad[e]:
        f = int(first[e])
        x = np.array([f], np.uint32).view(np.float32)[0]
        print(f"exp field {e:3d}: {int(bad[e]):10d} bad, first 0x{f:08x} = {x!r}")
