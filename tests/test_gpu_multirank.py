"""Multi-rank GPU rehearsal on ONE device: 2 ranks share cuda:0 over gloo.

RCCL refuses two ranks on one GPU, so this exercises everything of the N-GPU path
except the transport: sharded on-device data, HIP kernels per rank, collectives on
GPU tensors, rank-0 reporting and the bench JSON contract.

Default (``-m gpu``) cases never run a kernel that waits on another process's kernel:
the library sees that the ranks share one device (runtime.shared_device) and builds
no K11 exchange and no persistent / one-kernel K1 form. The K11 / persistent
rehearsals, which DO spin across processes on one GPU, are marked ``gpu_shared`` and
run only when DALGO_GPU_SHARED_TESTS=1 (own gpurun sessions, never the round-end tier).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, n=2, timeout=600, env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    return r.stdout


SCRIPTS = [
    ("optimization/bmuf.py", ["--synthetic", "50000,128", "--n-iterations", "5", "--quiet"], "Final acc:"),
    ("optimization/easgd.py", ["--synthetic", "50000,128", "--n-iterations", "5", "--quiet"], "Final acc:"),
    ("machine_learning/k-means.py", ["--synthetic", "20000,16", "--k", "8"], "Final centers:"),
    # bf16 d = 64: the Hamerly-bounded, incremental path on every rank
    ("machine_learning/k-means.py", ["--synthetic", "60000,64", "--k", "64", "--n-iterations", "6"],
     "Final centers:"),
    ("graph_computation/pagerank.py", ["--rmat-scale", "12", "--top", "3"], "has rank:"),
    ("matrix_computation/matrix_decomposition.py", [], "iterations: 4, rmse:"),
    ("randomized_algorithm/monte_carlo.py", ["--num-samples", "1000000"], "Pi is roughly"),
]


def test_scripts_two_ranks_gloo_on_one_gpu(cuda):
    """Every entry script with 2 gloo ranks on cuda:0, all in ONE torchrun job
    (tests/helpers/run_scripts.py: one process group, scripts run in-process in turn)."""
    jobs = [[p, ["--device", "cuda", "--backend", "gloo", "--no-plot"] + extra]
            for p, extra, _ in SCRIPTS]
    out = _torchrun(["tests/helpers/run_scripts.py", json.dumps(jobs)])
    for i, (path, _, needle) in enumerate(SCRIPTS):
        part = out.split(f"==BEGIN {i}==")[1].split(f"==END {i}==")[0]
        assert needle in part, (path, part[-2000:])


@pytest.mark.parametrize("n", [2, 3])
def test_pagerank_native_build_ranks(cuda, n):
    """The PageRank job at 2 and 3 gloo ranks on one GPU: every rank generates only its
    E / W input edges, the relabelled edges go to their destination owners in one
    all_to_all, each rank builds its K4b layout natively over the [own slice | ghosts]
    source space, runs the ghost exchange; the build witness checks every rank's edge set
    and out-degrees against torch over the whole raw input, and the ranks match the pull K4
    over the same edges."""
    out = _torchrun(["bench/pagerank_bench.py", "--gpus", str(n), "--backend", "gloo", "--scale", "15",
                     "--steps", "2", "--pool-gb", "1"], n=n)
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == n and d["exchange"] == "ghost"
    assert d["adjacency_build"].startswith("native") and "sharded" in d["adjacency_build"]
    w = d["correctness_witness"]
    assert w["passed"] and w["build"]["passed"] and w["build"]["edge_set_equal_rank0"], w


def test_bench_secondary_two_ranks(cuda):
    """bench.py at 2 gloo ranks on one GPU runs BASELINE configs #3-#5 too (reduced sizes):
    BMUF / EASGD, both k-means jobs and the sharded PageRank job, every witness passing."""
    out = _torchrun(["bench.py", "--gpus", "2", "--backend", "gloo", "--rows", "200000",
                     "--steps", "5", "--warmup", "2", "--secondary-steps", "5", "--secondary-warmup", "2",
                     "--km-rows", "2000000", "--pr-scale", "16", "--km-pool-gb", "4", "--pr-pool-gb", "4"])
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    sec = d["secondary"]
    assert set(sec) == {"bmuf", "easgd", "kmeans", "kmeans_overlapping", "pagerank"}, sec.keys()
    for k, v in sec.items():
        assert "error" not in v and "skipped" not in v, (k, v)
        assert v["correctness_witness"]["passed"], (k, v["correctness_witness"])
    assert sec["pagerank"]["n_gpus"] == 2 and "sharded" in sec["pagerank"]["adjacency_build"]


SPIN = {"DALGO_ALLOW_SHARED_SPIN": "1"}


def test_bench_two_ranks_shared_gpu(cuda):
    """bench.py with two gloo ranks on one GPU: one JSON line with the dp2 contract; every
    rank sees shared_device, K11 is never built even when forced (so no persistent /
    one-kernel form either) and the bench reports the process group."""
    out = _torchrun(["bench.py", "--gpus", "2", "--backend", "gloo", "--rows", "200000",
                     "--steps", "5", "--warmup", "2"], env_extra={"DALGO_XGMI": "1"})
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["value"] > 0
    assert d["shared_device"] is True and d["distinct_devices"] == 1
    assert d["config"]["allreduce"] == "gloo" and d["config"]["launch"] == "per-step"
    assert d["correctness_witness"]["passed"]


@pytest.mark.gpu_shared
@pytest.mark.parametrize("n", [2, 4, 8])
def test_xgmi_allreduce_ranks_on_one_gpu(cuda, n):
    """K11: IPC exchange buffers + flag protocol, exact rank-ordered sums on every rank."""
    out = _torchrun(["tests/helpers/xgmi_check.py"], n=n, env_extra=SPIN)
    assert f"XGMI_OK world={n}" in out


@pytest.mark.gpu_shared
def test_xgmi_timeout_raises_on_every_rank(cuda):
    """A K11 peer wait that times out on rank 0 only: the collective check raises on
    both ranks and shutdown exits non-zero (no rank silently continues)."""
    env = dict(os.environ, PYTHONPATH=ROOT, **SPIN)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "tests/helpers/xgmi_timeout.py"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert "XG_RAISED rank 0" in out and "XG_RAISED rank 1" in out, out[-3000:]
    assert "XG_NO_RAISE" not in out and "XG_SHUTDOWN_RETURNED" not in out, out[-3000:]
    assert r.returncode != 0


def _final_w(out):
    import numpy as np
    txt = out.split("Final w:")[1].split("Final acc")[0]
    return np.array([float(v) for v in txt.replace("[", " ").replace("]", " ").split()])


@pytest.mark.gpu_shared
@pytest.mark.parametrize("one_kernel", ["1", "0", "persistent", "graph"])
@pytest.mark.parametrize("algo", ["ssgd", "logistic_regression"])
def test_fused_xgmi_update_matches_process_group(cuda, algo, one_kernel):
    """SSGD / full-batch GD: one-launch step (K1 tail: xGMI exchange + update), a
    persistent multi-step launch (every step's tail exchanges over K11), or K1 + K11 with
    the fused K8 == gloo all-reduce + separate K8."""
    import numpy as np
    script = "optimization/ssgd.py" if algo == "ssgd" else "machine_learning/logistic_regression.py"
    args = [script, "--device", "cuda", "--backend", "gloo", "--no-plot", "--quiet",
            "--synthetic", "40000,64", "--n-iterations", "30", "--dtype", "f32",
            "--eval-every", "10"]   # persistent mode: 10-step launches between evaluations
    if one_kernel == "graph":
        # K1 + K11 (device-resident epoch) captured once, replayed every step
        mode = {"DALGO_GRAPH": "1", "DALGO_ONE_KERNEL": "0"}
    elif one_kernel == "persistent":
        mode = {"DALGO_PERSISTENT": "1"}
    else:
        mode = {"DALGO_ONE_KERNEL": one_kernel}
    fused = _torchrun(args, env_extra=dict(SPIN, DALGO_XGMI="1", **mode))
    plain = _torchrun(args, env_extra={"DALGO_XGMI": "0"})
    wf, wp = _final_w(fused), _final_w(plain)
    assert wf.shape == wp.shape and np.allclose(wf, wp, rtol=1e-4, atol=1e-5), (wf[:5], wp[:5])


@pytest.mark.gpu_shared
def test_bench_launch_calibration_two_ranks(cuda):
    """bench.py --launch auto with the K11 exchange: the per-step, hipGraph-replay,
    one-kernel and persistent forms are each timed on both ranks and one is kept (same on every rank)."""
    out = _torchrun(["bench.py", "--gpus", "2", "--backend", "gloo", "--rows", "200000",
                     "--steps", "5", "--warmup", "2", "--cal-steps", "4"],
                    env_extra=dict(SPIN, DALGO_XGMI="1"))
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    cal = d["launch_calibration_ms_per_step"]
    assert set(cal) == {"per-step", "graph", "one-kernel", "persistent"}
    assert d["config"]["launch"] == min(cal, key=cal.get)
    assert d["config"]["allreduce"] == "xgmi-oneshot (K11)" and d["value"] > 0


@pytest.mark.gpu_shared
def test_bench_auto_selects_allreduce(cuda):
    """DALGO_XGMI=auto (default): the start-up race picks a path and reports it."""
    out = _torchrun(["bench.py", "--gpus", "2", "--backend", "gloo", "--rows", "200000",
                     "--steps", "5", "--warmup", "2"], env_extra=SPIN)
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["config"]["allreduce"] in ("xgmi-oneshot (K11)", "gloo")


@pytest.mark.gpu_shared
def test_bench_eight_ranks_on_one_gpu(cuda):
    """World size 8 (the driver's largest N), 8 ranks sharing cuda:0: sharding of the
    10M-row global set into 1.25M-row shards, the 8-peer K11 exchange (or gloo if the
    start-up race prefers it), rank-0 JSON with the whole-job aggregate."""
    # (secondaries off: 8 spinning processes on one GPU run a step in ~90 ms, so the LR
    # witnesses' 1500-3000 training rounds alone would take minutes, profiles/round6/r6_61;
    # test_bench_secondary_two_ranks covers BASELINE configs #3-#5 on several ranks)
    out = _torchrun(["bench.py", "--gpus", "8", "--backend", "gloo", "--rows", "400000",
                     "--steps", "5", "--warmup", "2", "--secondary", "off"], n=8, env_extra=SPIN)
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 8 and d["steps"] == 5 and d["config"]["parallelism"] == "dp8"
    assert d["config"]["allreduce"] in ("xgmi-oneshot (K11)", "gloo")
    assert d["value"] > 0 and d["ms_per_step"] > 0
