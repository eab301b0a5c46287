"""Entry logic shared by the five logistic-regression scripts.

optimization/ssgd.py, optimization/ma.py, optimization/bmuf.py,
optimization/easgd.py and machine_learning/logistic_regression.py call
``main(algo)``. Defaults are the reference's module constants; stdout lines
and the PNG name match the reference scripts (rank 0 prints).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from dalgo.data.datasets import breast_cancer, synthetic_logistic
from dalgo.models.localsgd import ParallelSGD, SGDConfig
from dalgo.parallel import runtime
from dalgo.parallel.sharding import make_layout
from dalgo.utils import checkpoint, obs
from dalgo.utils.cli import common_parser, default_dtype, init_from_args

DEFAULTS = {
    # algo: (n_iterations, app name, plot file)            reference lines
    "ssgd": (1500, "SSGD", "ssgd_acc_plot.png"),           # ssgd.py:18,80,66
    "ma": (300, "Model Average", "ma_acc_plot.png"),       # ma.py:20
    "bmuf": (300, "BMUF", "bmuf_acc_plot.png"),            # bmuf.py:20
    "easgd": (1500, "EASGD", "easgd_acc_plot.png"),        # easgd.py:20
    "gd": (1500, "Logistic Regression", "logistic_regression_acc_plot.png"),
}


def build_parser(algo: str):
    n_it, name, _ = DEFAULTS[algo]
    ap = common_parser(f"{name} logistic regression (MI355X-native)")
    ap.add_argument("--n-slices", type=int, default=4, help="logical workers (n_slices)")
    ap.add_argument("--n-iterations", type=int, default=n_it)
    ap.add_argument("--eta", type=float, default=0.1)
    ap.add_argument("--mini-batch-fraction", type=float, default=0.1)
    ap.add_argument("--lam", type=float, default=0.0)
    ap.add_argument("--reg", default="l2", choices=["none", "l2", "l1", "elastic_net"])
    ap.add_argument("--n-local-iterations", type=int, default=5)
    ap.add_argument("--mu", type=float, default=0.9)
    ap.add_argument("--zeta", type=float, default=0.1)
    ap.add_argument("--rho", type=float, default=0.1)
    ap.add_argument("--sample-seed", type=int, default=42, help="sample(False, f, 42 + t)")
    ap.add_argument("--synthetic", default=None, metavar="N,D",
                    help="synthetic planted-logistic data instead of breast cancer")
    ap.add_argument("--dtype", choices=["bf16", "f32", "f64"], default=None,
                    help="feature storage dtype (default f32 on GPU, f64 on CPU)")
    ap.add_argument("--eval-every", type=int, default=1)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="hipGraph replay of whole steps (auto: MA/BMUF/EASGD on one rank)")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--resume", action="store_true")
    return ap


def main(algo: str, argv=None):
    a = build_parser(algo).parse_args(argv)
    _, name, plot = DEFAULTS[algo]
    rt = init_from_args(a, name)
    dtype = default_dtype(rt, a.dtype)
    model_dtype = torch.float32 if rt.device.type == "cuda" else torch.float64
    if rt.device.type == "cuda" and dtype == torch.float64:
        dtype = torch.float32
    P = a.n_slices
    if P % rt.world_size:
        P = rt.world_size * max(1, P // rt.world_size)
    if a.synthetic:
        N, D = (int(x) for x in a.synthetic.split(","))
        layout = make_layout(N, P, rt.world_size, rt.rank, spark_compatible=False)
        data = synthetic_logistic(N, D, row_range=(layout.row_lo, layout.row_hi),
                                  n_test=min(100_000, max(1000, N // 10)), device=rt.device,
                                  dtype=dtype, seed=a.seed + 1234)
    else:
        n_train = 398   # 569 * 0.7 (train_test_split(test_size=0.3)), ssgd.py:74-76
        layout = make_layout(n_train, P, rt.world_size, rt.rank)
        data = breast_cancer(device=rt.device, dtype=dtype, row_range=(layout.row_lo, layout.row_hi))
    cfg = SGDConfig(algo=algo, n_workers=P, n_iterations=a.n_iterations, eta=a.eta,
                    frac=a.mini_batch_fraction, lam=a.lam, reg=a.reg,
                    n_local=a.n_local_iterations, mu=a.mu, zeta=a.zeta, rho=a.rho,
                    sample_seed=a.sample_seed, init_seed=a.seed, eval_every=a.eval_every)
    model = ParallelSGD(cfg, data, layout, rt, model_dtype=model_dtype)
    if a.graph != "auto":
        model.graph = a.graph == "on"
    sink = obs.MetricsSink(a.metrics_out, rt.rank)
    if sink.enabled or obs.roctx_enabled():
        model.timer = obs.PhaseTimer(rt.device)
    ck_name = f"{algo}_state"
    if a.resume and a.ckpt_dir:
        sd = checkpoint.load(a.ckpt_dir, ck_name, rt.rank, per_rank=True)
        if sd is not None:
            model.load_state_dict(sd)
            rt.log(f"Resumed from iteration {model.t}")
    np.set_printoptions(precision=8)
    rt.log("Initial w: " + str(model.weights().double().cpu().numpy()))
    t0 = time.time()
    remaining = max(0, cfg.n_iterations - model.t)

    def cb(m):
        if sink.enabled:
            rec = dict(algo=algo, iteration=m.t, elapsed_s=time.time() - t0,
                       bytes_allreduced=m.bytes_allreduced, world_size=rt.world_size)
            if m.history.accs and m.history.iters[-1] == m.t:
                rec.update(accuracy=m.history.accs[-1], loss=m.history.losses[-1])
            sink.log(phases=m.timer.take(), **rec)
        elif m.timer is not None:
            m.timer.take()
        if a.ckpt_dir and a.ckpt_every and m.t % a.ckpt_every == 0:
            checkpoint.save(m.state_dict(), a.ckpt_dir, ck_name, rt.rank, per_rank=True)

    runtime.test_hang_point("fit")
    model.fit(remaining, verbose=not a.quiet, callback=cb)
    acc, _ = model.evaluate()
    rt.log("Final w: %s " % model.weights().double().cpu().numpy())
    rt.log("Final acc: %f" % acc)
    if a.ckpt_dir:
        checkpoint.save(model.state_dict(), a.ckpt_dir, ck_name, rt.rank, per_rank=True)
    if rt.is_main and not a.no_plot and model.history.accs:
        obs.draw_acc_plot(model.history.accs, plot)
    sink.close()
    runtime.shutdown()
    return acc
