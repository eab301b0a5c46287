"""Diagnostic: the (u, l) bounds after iteration 3 of the k-means job, dense filtered K2 vs
the drift-aware candidate K2 in that iteration (same state before it): where does the
next filter lose rows?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.data.synthetic import blobs  # noqa: E402
from dalgo.models.kmeans import KMeans, KMeansConfig  # noqa: E402
from dalgo.ops import kmeans as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
dev = torch.device("cuda")
X = blobs(n, 128, 1024, device=dev, dtype=torch.bfloat16, seed=7, noise=1.0)
res = {}
for name, fr in (("dense3", "0.4"), ("drift3", "0.75")):
    os.environ["DALGO_KM_DENSE_FRACTION"] = fr
    km = KMeans(KMeansConfig(k=1024, n_iterations=5, seed=1), X, 0, n)
    for _ in range(3):
        km.step()
    torch.cuda.synchronize()
    res[name] = (km._ul.clone(), km.assign.clone(), km.cen.Cq.clone())
    # what the next filter would do
    delta, s = K.centre_bounds(km.cen.Cq, km._cq_prev, 1024, 128)
    km2 = None
    print(name, "hist", km.active_history, flush=True)
    del km
ua, aa, ca = res["dense3"]
ub, ab, cb = res["drift3"]
print("assign equal:", bool(torch.equal(aa, ab)), "centres equal:", bool(torch.equal(ca, cb)))
du = (ub[:, 0] - ua[:, 0])
dl = (ub[:, 1] - ua[:, 1])
print("u: drift - dense  mean %.4f max %.4f" % (float(du.mean()), float(du.abs().max())))
print("l: drift - dense  mean %.4f  frac(l looser by >1) %.4f  by >10 %.4f" % (
    float(dl.mean()), float((dl < -1).float().mean()), float((dl < -10).float().mean())))
for lo, hi in ((0, 12), (12, 30), (30, 60), (60, 1e9)):
    m = (ua[:, 0] >= lo) & (ua[:, 0] < hi)
    if m.any():
        print(f"  u in [{lo},{hi}): rows {int(m.sum())}  l dense mean {float(ua[m,1].mean()):.1f}  "
              f"l drift mean {float(ub[m,1].mean()):.1f}  looser>10: {float((dl[m] < -10).float().mean()):.3f}")
