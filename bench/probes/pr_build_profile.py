"""Host-side profile of the native PageRank adjacency build (dalgo.ops.graph.build_native):
one warm build at a small scale, then cProfile around one build at the benchmark scale
with a device sync after every torch / extension call attributed to the caller line
(DALGO_BUILD_SYNC=1 phase marks). Prints the top functions by cumulative time."""
import argparse
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dalgo.apps.pagerank_app import build_rmat_native, rmat_input   # noqa: E402
from dalgo.ops import graph as G                                     # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=26)
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
dev = torch.device("cuda")
we, _ = rmat_input(16, 16, dev, seed=2)
build_rmat_native(we, 16, 0, 1, dev)
torch.cuda.synchronize()
edges, _ = rmat_input(a.scale, 16, dev, seed=1)
torch.cuda.synchronize()
G.build_marks = []
pr = cProfile.Profile()
pr.enable()
ng = build_rmat_native(edges, a.scale, 0, 1, dev)
torch.cuda.synchronize()
pr.disable()
print({k: round(v, 2) for k, v in G.build_phase_spans().items()})
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(a.top)
