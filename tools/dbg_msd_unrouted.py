import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle"); sys.path.insert(0, "/root/repo/tests")
import oracle as o
from orleans_amd import graindispatch as gd
from test_gpu_msd import _acts, _engine
n, n_act = 1 << 21, 300000
acts = _acts(n, n_act, "unrouted", 11)
e2 = _engine(gd, 2)
p2, off2 = e2.bucket(acts, n_act)
wp, wo = o.bucket_stable(acts, n_act)
bad = np.nonzero(p2 != wp)[0]
print("perm bad", len(bad), bad[:5], bad[-5:] if len(bad) else None)
print("off bad", np.nonzero(off2 != wo)[0][:10])
print("wo[n_act-2:]", wo[n_act-2:], "off2", off2[n_act-2:])
if len(bad):
    i = bad[0]; print("at", i, "got", p2[i:i+5], "want", wp[i:i+5], "acts(got)", acts[p2[i:i+5]], "acts(want)", acts[wp[i:i+5]])
