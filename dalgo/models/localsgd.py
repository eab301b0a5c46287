"""Parallel SGD for logistic regression: SSGD, full-batch GD, MA, BMUF, EASGD.

One scaffold for the reference's five LR-family scripts (optimization/ssgd.py,
optimization/ma.py, optimization/bmuf.py, optimization/easgd.py,
machine_learning/logistic_regression.py). The Spark driver loop becomes an SPMD
loop executed identically on every rank:

  SSGD / GD (ssgd.py:93-105, logistic_regression.py:76-85)
      K1+K7 fused sampled gradient  ->  all_reduce([g || count])  ->  K8 update
  MA / BMUF (ma.py:93-106, bmuf.py:98-114)
      reset locals to w (ma.py:96) -> n_local x [K1 on the SAME minibatch (seed 42+t
      is constant inside a round, ma.py:99) -> K8 local step] -> sum locals ->
      all_reduce -> K8 average / block-momentum rule
  EASGD (easgd.py:95-106)
      K1 -> K8 elastic local step (pull toward the old centre) -> sum locals ->
      all_reduce -> K8 centre update with the NEW locals (sequential, as the reference)

Logical workers (``n_workers`` = the reference's ``n_slices``) keep their Spark
partition rows (99/99/99/101 on breast cancer) and are spread over the ranks, so
a W-rank run and a 1-rank run with the same P compute the same thing. Each rank
holds only its rows (HBM-resident shard); the model and all sync state are
replicated, so no driver and no broadcast per iteration.
"""
from __future__ import annotations

import math
import os
from dataclasses import asdict, dataclass, field

import torch

from dalgo.data.datasets import LRData
from dalgo.ops import lr as lr_ops
from dalgo.ops import update as U
from dalgo.parallel import comm
from dalgo.parallel.runtime import Runtime
from dalgo.parallel.sharding import ShardLayout
from dalgo.utils.obs import NULL_PHASE

ALGOS = ("ssgd", "gd", "ma", "bmuf", "easgd")


@dataclass
class SGDConfig:
    algo: str = "ssgd"
    n_workers: int = 4            # n_slices (ssgd.py:17)
    n_iterations: int = 1500      # ssgd.py:18 (ma/bmuf: 300)
    eta: float = 0.1              # ssgd.py:19
    frac: float = 0.1             # mini_batch_fraction (ssgd.py:20)
    lam: float = 0.0              # ssgd.py:21
    reg: str = "l2"               # reg_gradient(w, "l2") at ssgd.py:105
    reg_alpha: float = 0.0
    n_local: int = 5              # ma.py:23
    mu: float = 0.9               # bmuf.py:24
    zeta: float = 0.1             # bmuf.py:25
    rho: float = 0.1              # easgd.py:23 (alpha = eta*rho, beta = P*alpha)
    eps: float | None = None      # sigmoid epsilon: 0 (ssgd/gd) or 1e-6 (ma/bmuf/easgd)
    sample_seed: int = 42         # sample(False, f, 42 + t)
    init_seed: int = 0            # the reference's np.random.ranf is unseeded
    reuse_minibatch: bool = True  # MA/BMUF: same sample for all local steps (ma.py:99)
    eval_every: int = 1           # test accuracy every k rounds (0 = never)
    # EASGD on several ranks: the centre all-reduce of round t runs (async, on the
    # collective stream) under the gradient kernel of round t+1, which does not read the
    # centre; the centre update is applied right before the elastic step that needs it
    overlap_center: bool = True

    def __post_init__(self):
        if self.algo not in ALGOS:
            raise ValueError(f"algo must be one of {ALGOS}")
        if self.eps is None:
            self.eps = 1e-6 if self.algo in ("ma", "bmuf", "easgd") else 0.0
        if self.algo == "gd":
            self.frac = 1.0

    @property
    def alpha(self) -> float:
        return self.eta * self.rho

    @property
    def beta(self) -> float:
        return self.n_workers * self.alpha


@dataclass
class TrainHistory:
    accs: list = field(default_factory=list)
    losses: list = field(default_factory=list)
    iters: list = field(default_factory=list)


def init_models(cfg: SGDConfig, ldw: int, dtype=torch.float64):
    """Deterministic stand-in for the reference's unseeded U[-1, 1) draws.

    Draw order follows the scripts: local models (ma.py:86), then w (ma.py:89),
    then BMUF's delta_w (bmuf.py:95).
    """
    g = torch.Generator().manual_seed(cfg.init_seed)
    out = {}
    if cfg.algo in ("ma", "bmuf", "easgd"):
        out["locals"] = 2 * torch.rand((cfg.n_workers, ldw), generator=g, dtype=dtype) - 1
    out["w"] = 2 * torch.rand(ldw, generator=g, dtype=dtype) - 1
    if cfg.algo == "bmuf":
        out["delta"] = 2 * torch.rand(ldw, generator=g, dtype=dtype) - 1
    return out


# DALGO_GRAPH=auto replays steps as a hipGraph only while the local shard is at most
# this large (launch-bound regime; see ParallelSGD._graph_ok)
_GRAPH_AUTO_MAX_BYTES = int(os.environ.get("DALGO_GRAPH_AUTO_MAX_MB", "256")) << 20


class ParallelSGD:
    def __init__(self, cfg: SGDConfig, data: LRData, layout: ShardLayout, rt: Runtime,
                 model_dtype: torch.dtype = torch.float32):
        self.cfg = cfg
        self.data = data
        self.layout = layout
        self.rt = rt
        dev = data.X_train.device
        self.device = dev
        if dev.type == "cuda" and model_dtype != torch.float32:
            raise ValueError("GPU kernels keep f32 master weights")
        self.D = data.D
        self.ldw = self.D + 1
        self.t = 0
        self.history = TrainHistory()
        P = cfg.n_workers
        init = init_models(cfg, self.ldw)
        self.w = init["w"].to(model_dtype).to(dev).view(1, -1).contiguous()
        algo = cfg.algo
        segs = layout.local_segments()
        if algo in ("ssgd", "gd"):
            self.seg = torch.tensor([0, layout.local_rows], dtype=torch.int64, device=dev)
            self.max_seg = layout.local_rows
            # fused all-reduce bucket [g (ldw) || count (1)]
            self.bucket = comm.BucketedAllReduce([(1, self.ldw), (1,)], dtype=model_dtype, device=dev)
            self.G, self.C = self.bucket.views
        else:
            self.seg = torch.tensor(segs, dtype=torch.int64, device=dev)
            self.max_seg = max(segs[i + 1] - segs[i] for i in range(len(segs) - 1))
            lo, hi = layout.worker_lo, layout.worker_hi
            self.W = init["locals"][lo:hi].to(model_dtype).to(dev).contiguous()
            self.G = torch.zeros((hi - lo, self.ldw), dtype=model_dtype, device=dev)
            self.C = torch.zeros(hi - lo, dtype=model_dtype, device=dev)
            self.S = torch.zeros(self.ldw, dtype=model_dtype, device=dev)
            if algo == "bmuf":
                self.Dl = init["delta"].to(model_dtype).to(dev).contiguous()
        self.inv_p = 1.0 / P
        # optional f64 device accumulator of minibatch sizes (bench accounting);
        # read it through global_sample_count()
        self.count_acc: torch.Tensor | None = None
        # G/C are zero (fresh, or left zeroed by the last gradient-consuming K8), so the
        # next atomic-epilogue K1 can accumulate into them without a memset launch
        self._g_zero = True
        self._zg = not lr_ops.DETERMINISTIC   # deterministic K1 overwrites G: no need to clear
        # hipGraph replay state (see _graph_ok): None = follow DALGO_GRAPH
        self.graph: bool | None = None
        self._graphs: dict = {}
        self._graph_warm = False
        self._t_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self._t_dev_val = 0
        self._upd = dict(mode=0 if algo == "ssgd" else 1, reg=U.REG.get(cfg.reg, 0), eta=cfg.eta,
                         lam=cfg.lam, reg_alpha=cfg.reg_alpha)
        # observability (dalgo.utils.obs.PhaseTimer; None = off, no per-step cost) and
        # the running count of bytes this rank all-reduced
        self.timer = None
        self.bytes_allreduced = 0
        ar = self.bucket.buffer if algo in ("ssgd", "gd") else self.S
        self._ar_bytes = ar.numel() * ar.element_size()

    def _ph(self, name: str):
        return self.timer.phase(name) if self.timer is not None else NULL_PHASE

    def _count_ar(self, n: int = 1):
        if comm.world_size() > 1:
            self.bytes_allreduced += n * self._ar_bytes

    # ------------------------------------------------------------------ steps
    def _grad(self, W, stream, step_dev=None, step_mul=1):
        c = self.cfg
        lr_ops.lr_grad(self.data.X_train, self.data.y_train, W, self.seg, D=self.D, has_bias=True,
                       eps=c.eps, seed=c.sample_seed, step=stream, frac=c.frac,
                       row_offset=self.data.row_offset, G=self.G, C=self.C,
                       max_seg_rows=self.max_seg, g_is_zero=self._g_zero,
                       step_dev=step_dev, step_mul=step_mul)
        self._g_zero = False

    def _one_kernel(self) -> bool:
        """Fused single-launch step (DALGO_ONE_KERNEL=1): GPU, atomic epilogue, one rank or
        K11 peers. Measured on MI355X equal to K1 + separate update / K11 launch (361 vs
        361 us at 10M rows, 59.1 vs 59.7 us at 1.25M, 76.7 vs 76.5 us for 2 ranks on one
        GPU): back-to-back launches already overlap, and the last-block hand-off adds the
        latency the launch saves. Off by default; kept tested."""
        if getattr(self, "_ok1", None) is None:
            self._ok1 = (self.device.type == "cuda" and self._zg
                         and os.environ.get("DALGO_ONE_KERNEL", "0") == "1"
                         and (comm.world_size() == 1 or self.bucket.xg is not None))
        return self._ok1

    def _persistent(self) -> bool:
        """Persistent multi-step launches (DALGO_PERSISTENT=1): SSGD / GD on GPU, atomic
        epilogue, one rank or K11 peers. K steps run as ONE cooperative K1 grid whose tail
        block releases each step's model (csrc/kernels/lr_grad.hip, nsteps)."""
        if getattr(self, "_okp", None) is None:
            self._okp = (self.device.type == "cuda" and self._zg
                         and self.cfg.algo in ("ssgd", "gd")
                         and os.environ.get("DALGO_PERSISTENT", "0") == "1"
                         and (comm.world_size() == 1 or self.bucket.xg is not None))
        return self._okp

    def run_steps(self, k: int):
        """k training steps (one persistent launch when enabled, else k step() calls)."""
        k = int(k)
        if k <= 0:
            return
        if not self._persistent():
            for _ in range(k):
                self.step()
            return
        c = self.cfg
        with self._ph("persistent_launch"):
            lr_ops.lr_grad(self.data.X_train, self.data.y_train, self.w, self.seg, D=self.D,
                           has_bias=True, eps=c.eps, seed=c.sample_seed, step=self.t, frac=c.frac,
                           row_offset=self.data.row_offset, G=self.G, C=self.C,
                           max_seg_rows=self.max_seg, g_is_zero=self._g_zero,
                           tail=dict(mode=0 if c.algo == "ssgd" else 1, reg=self._upd["reg"],
                                     eta=c.eta, lam=c.lam, reg_alpha=c.reg_alpha,
                                     count_acc=self.count_acc, xg=self.bucket.xg, nsteps=k))
        self._count_ar(k)
        self._g_zero = True
        self.t += k

    def global_sample_count(self) -> float:
        """Total minibatch rows accumulated in count_acc, summed over ranks (exact, counted
        on the device). SSGD / GD count the all-reduced minibatch once per step; MA / BMUF
        / EASGD count every local model's minibatch at every local step (the gradient rows
        actually processed: ma.py:98-102 re-reads the same sample n_local times)."""
        if self.count_acc is None:
            return 0.0
        cnt = self.count_acc.clone()
        if self.cfg.algo in ("ma", "bmuf", "easgd"):
            comm.all_reduce_sum(cnt)   # these kernels accumulate LOCAL counts
        return float(cnt.item())

    # ------------------------------------------------------- hipGraph replay
    def _graph_ok(self) -> bool:
        """Replay whole training steps from one captured hipGraph (DALGO_GRAPH=1 or auto,
        or ``model.graph = True``). Every kernel of a step (K1 gradient, K8 updates, row
        sums, the model all-reduce) is recorded once; the sampling stream comes from a
        device step counter (K1 ``step_dev``) that the graph itself advances, so a replay
        is one host call per step instead of 2 (SSGD) to 14 (MA/BMUF, 5 local steps)
        launches. Needs GPU tensors, no persistent / one-kernel mode, and capturable
        collectives: one rank, RCCL, or the K11 xGMI exchange (its epoch lives on the
        device and is advanced by the kernel itself, csrc/include/dalgo/xgmi.h)."""
        if getattr(self, "_okg", None) is None:
            ws = comm.world_size()
            env = os.environ.get("DALGO_GRAPH", "auto")
            # auto: the multi-launch MA / BMUF / EASGD steps on one rank while they are
            # launch bound (measured 1.05-1.8x faster replayed up to 100k x 256 bf16,
            # bench/graph_replay.py; 5-7% SLOWER at 10M x 1024, where back-to-back eager
            # launches overlap better than graph nodes); SSGD / GD (two launches) stay
            # eager (0.75-0.9x replayed)
            X = self.data.X_train
            small = X.numel() * X.element_size() <= _GRAPH_AUTO_MAX_BYTES
            auto = self.cfg.algo in ("ma", "bmuf", "easgd") and ws == 1 and small
            want = self.graph if self.graph is not None else (
                env == "1" or (env == "auto" and auto))
            # capturable collectives: RCCL, or every collective of the step through K11
            if self.cfg.algo in ("ssgd", "gd"):
                k11 = getattr(getattr(self, "bucket", None), "xg", None) is not None and self._zg
            else:
                k11 = self.device.type == "cuda" and comm.uses_xgmi(self.S)
            ok_comm = ws == 1 or k11 or torch.distributed.get_backend() == "nccl"
            self._okg = bool(want and self.device.type == "cuda"
                             and not self._persistent() and not self._one_kernel() and ok_comm)
        return self._okg

    def _graph_step(self):
        # count_acc's address is baked into the captured kernels: one graph per target
        key = None if self.count_acc is None else self.count_acc.data_ptr()
        g = self._graphs.get(key)
        if g is None:
            if not self._graph_warm:
                # one eager step allocates the kernel workspaces and reaches the
                # steady state (G / C zero between steps) the capture assumes
                self._step_impl(self.t)
                self.t += 1
                torch.cuda.synchronize(self.device)
                self._graph_warm = True
                return
            # a deferred EASGD centre update of the warm step must land before capture:
            # the captured step must not contain (or wait on) a collective issued eagerly
            self._finish_center()
            g = torch.cuda.CUDAGraph()
            timer, self.timer = self.timer, None     # no timing events inside a capture
            ar = self.bytes_allreduced
            xg = comm.xgmi_instance()
            ex = xg.exchanges if xg is not None else 0
            try:
                # thread_local: the process group's watchdog thread keeps querying its own
                # streams during the capture, which a global-mode capture would reject
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self._step_impl(0, self._t_dev)
                    self._t_dev.add_(1)
            finally:
                self.timer = timer
            self._ar_per_replay = self.bytes_allreduced - ar
            self.bytes_allreduced = ar
            # K11 exchanges recorded in the graph (host epoch-space guard, per replay)
            self._ex_per_replay = (xg.exchanges - ex) if xg is not None else 0
            self._graphs[key] = g
        if self._t_dev_val != self.t:
            self._t_dev.fill_(self.t)
        with self._ph("step_graph"):
            g.replay()
        self.bytes_allreduced += getattr(self, "_ar_per_replay", 0)
        if getattr(self, "_ex_per_replay", 0):
            comm.xgmi_instance().count(self._ex_per_replay)
        self.t += 1
        self._t_dev_val = self.t

    def step(self):
        if self._graph_ok():
            self._graph_step()
            return
        self._step_impl(self.t)
        self.t += 1

    def _step_impl(self, t: int, step_dev: torch.Tensor | None = None):
        """One training step at sampling step t (or at the device counter step_dev);
        does not advance self.t."""
        c = self.cfg
        sd = dict(step_dev=step_dev) if step_dev is not None else {}
        if step_dev is not None:
            t = 0
        if c.algo in ("ssgd", "gd") and self._one_kernel():
            # the whole step in ONE launch: gradient, (xGMI exchange,) update
            self._count_ar()
            with self._ph("step_one_kernel"):
                lr_ops.lr_grad(self.data.X_train, self.data.y_train, self.w, self.seg, D=self.D,
                               has_bias=True, eps=c.eps, seed=c.sample_seed, step=t, frac=c.frac,
                               row_offset=self.data.row_offset, G=self.G, C=self.C,
                               max_seg_rows=self.max_seg, g_is_zero=self._g_zero,
                               tail=dict(mode=0 if c.algo == "ssgd" else 1, reg=self._upd["reg"],
                                         eta=c.eta, lam=c.lam, reg_alpha=c.reg_alpha,
                                         count_acc=self.count_acc, xg=self.bucket.xg))
            self._g_zero = True
        elif c.algo in ("ssgd", "gd"):
            with self._ph("sample+grad"):
                self._grad(self.w, t, **sd)
            xg = self.bucket.xg
            self._count_ar()
            if xg is not None and self._zg:
                # K11 all-reduce + K8 update in one launch; leaves the bucket zeroed
                with self._ph("allreduce+update"):
                    xg.all_reduce_update_(self.bucket.buffer, self.w,
                                          mode=0 if c.algo == "ssgd" else 1,
                                          reg=self._upd["reg"], eta=c.eta, lam=c.lam,
                                          reg_alpha=c.reg_alpha, count_index=self.ldw,
                                          count_acc=self.count_acc)
                self._g_zero = True
                return
            with self._ph("allreduce"):
                self.bucket.all_reduce()
            with self._ph("update"):
                if c.algo == "ssgd":
                    U.sync_update(self.w, U.SSGD, G=self.G, C=self.C, reg=c.reg, eta=c.eta,
                                  lam=c.lam, reg_alpha=c.reg_alpha, count_acc=self.count_acc,
                                  zero_grad=self._zg)
                else:
                    U.sync_update(self.w, U.GD_SUM, G=self.G, C=self.C, eta=c.eta,
                                  count_acc=self.count_acc, zero_grad=self._zg)
            self._g_zero = True
        elif c.algo in ("ma", "bmuf"):
            U.rows_broadcast(self.W, self.w)
            for l in range(c.n_local):
                stream = t if c.reuse_minibatch else t * c.n_local + l
                with self._ph("sample+grad"):
                    if step_dev is not None:
                        # stream = (0 | l) + (1 | n_local) * step_dev
                        self._grad(self.W, 0 if c.reuse_minibatch else l, step_dev,
                                   1 if c.reuse_minibatch else c.n_local)
                    else:
                        self._grad(self.W, stream)
                with self._ph("local_update"):
                    U.sync_update(self.W, U.LOCAL_MEAN, G=self.G, C=self.C, eta=c.eta,
                                  count_acc=self.count_acc, zero_grad=self._zg)
                self._g_zero = True
            with self._ph("allreduce"):
                U.rows_sum(self.W, self.S)
                comm.all_reduce_sum(self.S)
            self._count_ar()
            with self._ph("update"):
                if c.algo == "ma":
                    U.sync_update(self.w, U.AVERAGE, S=self.S, inv_p=self.inv_p)
                else:
                    U.sync_update(self.w, U.BMUF, S=self.S, Dl=self.Dl, mu=c.mu, zeta=c.zeta,
                                  inv_p=self.inv_p)
        else:  # easgd
            with self._ph("sample+grad"):
                self._grad(self.W, t, **sd)
            # the centre of this round = previous round's locals (easgd.py:104-106): its
            # all-reduce may still be in flight under the gradient kernel above
            self._finish_center()
            with self._ph("local_update"):
                U.sync_update(self.W, U.LOCAL_ELASTIC, G=self.G, C=self.C, center=self.w,
                              eta=c.eta, alpha=c.alpha, count_acc=self.count_acc,
                              zero_grad=self._zg)
            self._g_zero = True
            U.rows_sum(self.W, self.S)
            self._count_ar()
            if self._overlap_ok(step_dev):
                self._center_work = comm.all_reduce_sum(self.S, async_op=True)
            else:
                with self._ph("allreduce"):
                    comm.all_reduce_sum(self.S)
                with self._ph("update"):
                    U.sync_update(self.w, U.ELASTIC_CENTER, S=self.S, beta=c.beta,
                                  inv_p=self.inv_p)

    def _overlap_ok(self, step_dev=None) -> bool:
        """EASGD centre all-reduce deferred under the next gradient (several ranks, eager).

        Never under hipGraph replay (the captured step would consume a collective issued
        outside the graph) and never when the small-vector all-reduce goes through K11:
        the async form would route the centre through the process group instead of the
        one-shot exchange the start-up race chose."""
        if not (self.cfg.algo == "easgd" and self.cfg.overlap_center and comm.world_size() > 1
                and step_dev is None and os.environ.get("DALGO_EASGD_OVERLAP", "1") != "0"):
            return False
        if self._graph_ok():
            return False
        if self.device.type == "cuda":
            if torch.cuda.is_current_stream_capturing() or comm.uses_xgmi(self.S):
                return False
        return True

    def _finish_center(self):
        """Complete a deferred EASGD centre update: w = (1-beta) w + beta * sum(locals)/P."""
        work = getattr(self, "_center_work", None)
        if work is None:
            return
        self._center_work = None
        with self._ph("allreduce_wait"):
            work.wait()
        c = self.cfg
        with self._ph("update"):
            U.sync_update(self.w, U.ELASTIC_CENTER, S=self.S, beta=c.beta, inv_p=self.inv_p)

    def _maybe_check_errors(self, reported: bool):
        """Collective device-error check before an evaluation.

        ``reported``: the result is about to leave the process (printed, handed to a
        callback / metrics sink): always checked first, so no number computed after a
        timed-out device wait is ever shown as valid. Silent evaluations (history only,
        which fit() returns after its own end-of-fit check) are checked every 100th time:
        each check is a collective plus host syncs on a ~50 us step."""
        self._n_evals = getattr(self, "_n_evals", 0) + 1
        if reported or self._n_evals % 100 == 0:
            comm.check_device_errors("evaluation")

    def evaluate(self):
        self._finish_center()
        d = self.data
        if d.X_test.shape[0] == 0:
            return float("nan"), float("nan")
        with self._ph("eval"):
            correct, loss = lr_ops.lr_eval(d.X_test, d.y_test, self.w, D=self.D, has_bias=True,
                                           eps=self.cfg.eps)
        return int(correct.item()) / d.X_test.shape[0], float(loss.item())

    def fit(self, n_iterations: int | None = None, verbose: bool = False, callback=None):
        n = self.cfg.n_iterations if n_iterations is None else n_iterations
        acc = float("nan")
        if self._persistent() and not verbose:
            # persistent launches between evaluation points (the callback runs once per
            # launch, at the evaluation step)
            done = 0
            while done < n:
                ev = self.cfg.eval_every
                k = n - done if not ev else min(n - done, ev - self.t % ev)
                self.run_steps(k)
                done += k
                if ev and self.t % ev == 0:
                    self._maybe_check_errors(callback is not None)
                    acc, loss = self.evaluate()
                    self.history.accs.append(acc)
                    self.history.losses.append(loss)
                    self.history.iters.append(self.t)
                if callback is not None:
                    callback(self)
            comm.check_device_errors("end of fit")
            return self.history
        for _ in range(n):
            if verbose:
                self.rt.log("On iteration %d" % (self.t + 1))
            self.step()
            if self.cfg.eval_every and (self.t % self.cfg.eval_every == 0):
                self._maybe_check_errors(verbose or callback is not None)
                acc, loss = self.evaluate()
                self.history.accs.append(acc)
                self.history.losses.append(loss)
                self.history.iters.append(self.t)
                if verbose:
                    self.rt.log("iterations: %d, accuracy: %f" % (self.t - 1, acc))
            if callback is not None:
                callback(self)
        self._finish_center()
        comm.check_device_errors("end of fit")
        return self.history

    # --------------------------------------------------------- checkpointing
    def state_dict(self) -> dict:
        self._finish_center()
        # copy=True: on a CPU model .cpu() would alias the live tensors (a snapshot that
        # later training overwrites)
        sd = {"t": self.t, "w": self.w.detach().to("cpu", copy=True), "cfg": asdict(self.cfg),
              "accs": list(self.history.accs)}
        if hasattr(self, "W"):
            sd["locals"] = self.W.detach().to("cpu", copy=True)
            sd["worker_lo"] = self.layout.worker_lo
        if hasattr(self, "Dl"):
            sd["delta"] = self.Dl.detach().to("cpu", copy=True)
        return sd

    def load_state_dict(self, sd: dict):
        self.t = int(sd["t"])
        self.w.copy_(sd["w"].to(self.w.dtype))
        if "locals" in sd and hasattr(self, "W"):
            self.W.copy_(sd["locals"].to(self.W.dtype))
        if "delta" in sd and hasattr(self, "Dl"):
            self.Dl.copy_(sd["delta"].to(self.Dl.dtype))
        self.history.accs = list(sd.get("accs", []))

    def weights(self) -> torch.Tensor:
        self._finish_center()
        return self.w.view(-1)
