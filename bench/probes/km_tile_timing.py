"""Per-tile phase clocks of the candidate-pruned K2 (a build with -DKM_XP_TIMING, loaded
through DALGO_EXT_LIB): for the first 64 blocks x 64 tiles of the K2 launch of iteration
--at, the shader-clock time of each phase of a tile (wave 0):
  drain  tile start -> earlier memory ops retired (vmcnt(0), timing build only)
  load   -> point / set-up loads landed (prologue vmcnt(0))
  setup  -> tile distances, R, neighbour list staged (block barrier)
  c0     -> chunk 0 landed (its DMA is issued after the barrier)
  chunks -> last chunk's MFMAs and reductions done
  epi    -> epilogue (decode, bound / assign stores, moved-row buffer)
  gap    previous tile's end -> this tile's start
Timing only."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dalgo.data.synthetic import blobs          # noqa: E402
from dalgo.models.kmeans import KMeans, KMeansConfig   # noqa: E402
from dalgo.ops import kmeans as K               # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=50_000_000)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", default="2,4")
a = ap.parse_args()
lib = ctypes.CDLL(os.environ["DALGO_EXT_LIB"])
NB, NT, NS = 64, 64, 16
dev = torch.device("cuda")
X = blobs(a.rows, 128, a.k, device=dev, dtype=torch.bfloat16, seed=7)
km = KMeans(KMeansConfig(k=a.k, n_iterations=5, seed=42), X, 0, a.rows)
orig = K.assign_rows
want = {int(v) for v in a.iters.split(",")}
out = {}
calls = [0]


def probe(*args, post=None, cand=None, **kw):
    r = orig(*args, post=post, cand=cand, **kw)
    if post is not None and cand is not None:
        calls[0] += 1
        it = calls[0] + 1
        if it in want:
            torch.cuda.synchronize()
            buf = np.zeros(NB * NT * NS, dtype=np.uint64)
            rc = lib.dalgo_km_dbg_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
            assert rc == 0, rc
            b = buf.reshape(NB, NT, NS).astype(np.int64)
            ok = (b[:, :, 5] > 0) & (b[:, :, 0] > 0)
            ph = {"drain": b[:, :, 7] - b[:, :, 0], "load": b[:, :, 1] - b[:, :, 7],
                  "setup": b[:, :, 2] - b[:, :, 1],
                  "w_last_start": b[:, :, 8] - b[:, :, 0], "w_last_drain": b[:, :, 15] - b[:, :, 8],
                  "w_last_load": b[:, :, 9] - b[:, :, 15], "w_last_setup": b[:, :, 10] - b[:, :, 9],
                  "c0": b[:, :, 3] - b[:, :, 2], "chunks": b[:, :, 4] - b[:, :, 3],
                  "epi": b[:, :, 5] - b[:, :, 4]}
            gap = np.zeros_like(b[:, :, 0])
            gap[:, 1:] = b[:, 1:, 0] - b[:, :-1, 5]
            okg = ok.copy()
            okg[:, 0] = False
            okg[:, 1:] &= ok[:, :-1]
            res = {k2: float(np.median(v[ok])) for k2, v in ph.items()}
            res.update({k2 + "_mean": float(np.mean(v[ok])) for k2, v in ph.items()})
            res["gap"] = float(np.median(gap[okg]))
            res["gap_mean"] = float(np.mean(gap[okg]))
            nch = b[:, :, 6][ok]
            res["chunks_mean"] = float(nch.mean())
            res["cycles_per_chunk_mean"] = float((ph["chunks"][ok] / np.maximum(nch, 1)).mean())
            res["tiles_sampled"] = int(ok.sum())
            out[f"iteration_{it}"] = res
    return r


K.assign_rows = probe
for _ in range(max(want)):
    km.step()
print(json.dumps(out, indent=1))
