"""A/B of the filtered-iteration K2 forms on the same active rows (iteration 2 state of the
5-iteration benchmark job): Hamerly-only K2 on the filter's row order, the same kernel on
the cluster-sorted order, the candidate-pruned K2, and the candidate K2 forced to stream
every chunk (nd = 0). Timing only (each run rewrites assign / u / l)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from dalgo.data.synthetic import blobs          # noqa: E402
from dalgo.models.kmeans import KMeans, KMeansConfig   # noqa: E402
from dalgo.ops import kmeans as K               # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=50_000_000)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--at", type=int, default=2, help="iteration whose K2 is compared")
a = ap.parse_args()
dev = torch.device("cuda")
X = blobs(a.rows, 128, a.k, device=dev, dtype=torch.bfloat16, seed=7)
km = KMeans(KMeansConfig(k=a.k, n_iterations=5, seed=42), X, 0, a.rows)
orig = K.assign_rows
res = {}


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


calls = [0]


def probe(X_, cen, idx, m, assign, *args, post=None, cand=None, **kw):
    if post is not None:
        calls[0] += 1
        if calls[0] == a.at - 1:
            torch.cuda.synchronize()
            n_act = int(post["m_dev"].item())
            snap = {k2: v.clone() for k2, v in post.items() if isinstance(v, torch.Tensor)}
            asg = assign.clone()

            def restore():
                for k2, v in snap.items():
                    post[k2].copy_(v)
                assign.copy_(asg)
                post["n_changed"].zero_()
            idx_f = km._idx
            # the Hamerly-only form reads the previous clusters (the candidate form knows
            # them from its tile's cluster): the snapshot of assign is that
            post_h = dict(post, a_prev=asg, chg_new=None, chg_old=None)
            runs = {
                "hamerly_filter_order": lambda: orig(X_, cen, idx_f, m, assign, post=post_h),
                "hamerly_sorted_order": lambda: orig(X_, cen, cand.rows, m, assign, post=post_h),
                "candidates": lambda: orig(X_, cen, cand.rows, m, assign, post=post, cand=cand),
            }
            for name, fn in runs.items():
                restore()
                res[name] = timed(lambda: (restore(), fn()))
            nd0 = cand.nd.clone()
            cand.nd.zero_()
            restore()
            res["candidates_all_chunks"] = timed(lambda: (restore(), orig(X_, cen, cand.rows, m, assign, post=post, cand=cand)))
            cand.nd.copy_(nd0)
            restore()
            res["restore_only"] = timed(restore)
            # a standalone scatter of one 8-byte pair per active row (torch index_copy_)
            ul = post["ul"]
            src = torch.randn(n_act, 2, device=ul.device)
            rl = cand.rows[:n_act].long()
            res["scatter_pairs_torch"] = timed(lambda: ul.index_copy_(0, rl, src))
            rs = torch.sort(rl).values
            res["scatter_pairs_sorted_rows"] = timed(lambda: ul.index_copy_(0, rs, src))
            res["active"] = n_act
    return orig(X_, cen, idx, m, assign, *args, post=post, cand=cand, **kw)


K.assign_rows = probe
for it in range(a.at):
    km.step()
print(json.dumps(res))
