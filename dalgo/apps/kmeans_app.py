"""machine_learning/k-means.py entry logic (defaults = the reference constants)."""
from __future__ import annotations

import numpy as np
import torch

from dalgo.data.synthetic import blobs
from dalgo.models.kmeans import KMeans, KMeansConfig
from dalgo.parallel import comm, runtime
from dalgo.parallel.sharding import even_slices, spark_slices
from dalgo.utils import checkpoint, obs
from dalgo.utils.cli import add_ckpt_args, common_parser, init_from_args

TOY = [[1, 2], [1, 4], [1, 0], [10, 2], [10, 4], [10, 0]]   # k-means.py:49-50


def main(argv=None):
    ap = common_parser("Distributed Lloyd k-means (MI355X-native)")
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--n-iterations", type=int, default=5)
    ap.add_argument("--n-slices", type=int, default=2)
    ap.add_argument("--converge-dist", type=float, default=None,
                    help="stop when the squared centre shift < this (the reference declares convergeDist=0.1 but never uses it)")
    ap.add_argument("--init-seed", type=int, default=42, help="takeSample(False, k, 42)")
    ap.add_argument("--synthetic", default=None, metavar="N,D",
                    help="Gaussian blobs instead of the 6 toy points")
    ap.add_argument("--dtype", choices=["bf16", "f32"], default=None)
    add_ckpt_args(ap)
    a = ap.parse_args(argv)
    rt = init_from_args(a, "K-means")
    if a.synthetic:
        N, D = (int(x) for x in a.synthetic.split(","))
        lo, hi = even_slices(N, rt.world_size)[rt.rank]
        dtype = torch.bfloat16 if (a.dtype or ("bf16" if rt.device.type == "cuda" else "f32")) == "bf16" else torch.float32
        X = blobs(N, D, a.k, row_range=(lo, hi), device=rt.device, dtype=dtype, seed=a.seed + 99)
    else:
        N = len(TOY)
        slices = spark_slices(N, max(a.n_slices, rt.world_size))
        per = len(slices) // rt.world_size
        lo, hi = slices[rt.rank * per][0], slices[(rt.rank + 1) * per - 1][1]
        X = torch.tensor(TOY[lo:hi], dtype=torch.float32, device=rt.device)
    cfg = KMeansConfig(k=a.k, n_iterations=a.n_iterations, n_workers=a.n_slices, seed=a.init_seed,
                       tol=a.converge_dist)
    km = KMeans(cfg, X, lo, N)
    if a.resume and a.ckpt_dir:
        sd = checkpoint.load(a.ckpt_dir, "kmeans_state")
        if sd is not None:
            km.load_state_dict(sd)
            rt.log(f"Resumed from iteration {km.t}")
    sink = obs.MetricsSink(a.metrics_out, rt.rank)
    if sink.enabled or obs.roctx_enabled():
        km.timer = obs.PhaseTimer(rt.device)
    while km.t < a.n_iterations:
        km.fit(1)
        sink.log(phases=km.timer.take() if km.timer else None, iteration=km.t,
                 sse=km.history.sse[-1], shift2=km.history.shift[-1],
                 bytes_allreduced=km.bytes_allreduced, world_size=rt.world_size)
        if a.ckpt_dir and a.ckpt_every and km.t % a.ckpt_every == 0:
            checkpoint.save(km.state_dict(), a.ckpt_dir, "kmeans_state", rt.rank)
        if cfg.tol is not None and km.history.shift and km.history.shift[-1] < cfg.tol:
            break
    C = km.centers.cpu().numpy()
    rt.log("Final centers: " + str([np.array(c) for c in C]))
    if a.ckpt_dir:
        checkpoint.save(km.state_dict(), a.ckpt_dir, "kmeans_state", rt.rank)
    if X.shape[1] == 2 and not a.no_plot:
        counts = [hi - lo] if rt.world_size == 1 else None
        if rt.world_size > 1:
            cnt = torch.tensor([hi - lo], device=rt.device)
            allc = torch.zeros(rt.world_size, dtype=cnt.dtype, device=rt.device)
            comm.all_gather_into(allc, cnt)
            counts = allc.tolist()
        pts = comm.all_gather_varlen(X.float(), counts)
        asg = comm.all_gather_varlen(km.predict(X).view(-1, 1), counts).view(-1)
        if rt.is_main:
            obs.display_clusters(pts.cpu().numpy(), asg.cpu().numpy(), a.k, "kmeans_clusters_display.png")
    sink.close()
    runtime.shutdown()
    return C
