"""The reference-path entry scripts run end-to-end (CPU) and print the reference lines."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT
    env.update(env_extra or {})
    r = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("script,needle", [
    ("optimization/ssgd.py", "Final acc:"),
    ("optimization/ma.py", "Final acc:"),
    ("optimization/bmuf.py", "Final acc:"),
    ("optimization/easgd.py", "Final acc:"),
    ("machine_learning/logistic_regression.py", "Final acc:"),
])
def test_lr_scripts(script, needle, tmp_path):
    out = _run([script, "--device", "cpu", "--n-iterations", "30", "--quiet", "--no-plot",
                "--metrics-out", str(tmp_path / "m.jsonl")])
    assert "Initial w:" in out and needle in out
    lines = (tmp_path / "m.jsonl").read_text().splitlines()
    assert len(lines) == 30 and "accuracy" in json.loads(lines[-1])


def test_kmeans_script():
    out = _run(["machine_learning/k-means.py", "--device", "cpu", "--no-plot"])
    assert "Final centers: [array([1., 2.]" in out and "array([10.,  2.]" in out


def test_pagerank_script():
    out = _run(["graph_computation/pagerank.py", "--device", "cpu"])
    assert "1 has rank: 0.38891305880091237." in out
    assert "2 has rank: 0.214416470596171." in out
    assert "3 has rank: 0.3966704706029163." in out


def test_closure_script():
    out = _run(["graph_computation/transitive_closure.py", "--device", "cpu"])
    assert "The original graph has 9 paths" in out


@pytest.mark.parametrize("engine", ["dense", "sparse"])
def test_closure_checkpoint_resume(engine, tmp_path):
    """Stop after 2 join rounds with a checkpoint, resume: same fixpoint and per-round
    count trajectory as an uninterrupted run."""
    base = ["graph_computation/transitive_closure.py", "--device", "cpu", "--engine", engine,
            "--random", "300,420", "--seed", "3"]
    full = _run(base)
    ck = ["--ckpt-dir", str(tmp_path)]
    part = _run(base + ck + ["--max-rounds", "2"])
    assert "before the fixpoint" in part
    res = _run(base + ck + ["--resume"])
    assert "resumed after 2 rounds" in res
    traj = [l for l in full.splitlines() if l.startswith("path counts per round")]
    assert traj and traj == [l for l in res.splitlines() if l.startswith("path counts per round")]
    final = [l for l in full.splitlines() if "The original graph has" in l]
    assert final == [l for l in res.splitlines() if "The original graph has" in l]


def test_closure_resume_two_ranks_gloo(tmp_path):
    """Per-rank closure checkpoints (each rank owns its target slice) at 2 gloo ranks."""
    tr = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
          "--master-addr", "127.0.0.1"]
    base = ["graph_computation/transitive_closure.py", "--device", "cpu", "--backend", "gloo",
            "--engine", "sparse", "--random", "200,300", "--seed", "5", "--ckpt-dir", str(tmp_path)]
    full = _run(["graph_computation/transitive_closure.py", "--device", "cpu", "--engine", "sparse",
                 "--random", "200,300", "--seed", "5"])
    _run(tr + ["--master-port", str(_port())] + base + ["--max-rounds", "3"], timeout=400)
    assert sorted(os.listdir(tmp_path)) == ["closure_sparse_w2.rank0.pt", "closure_sparse_w2.rank1.pt"]
    res = _run(tr + ["--master-port", str(_port())] + base + ["--resume"], timeout=400)
    final = [l for l in full.splitlines() if "The original graph has" in l]
    assert final and final == [l for l in res.splitlines() if "The original graph has" in l]

    # a missing per-rank file, or a checkpoint of another graph: every rank refuses
    bad = tmp_path / "bad"
    bad.mkdir()
    import shutil
    shutil.copy(tmp_path / "closure_sparse_w2.rank0.pt", bad / "closure_sparse_w2.rank0.pt")
    base_bad = [x if x != str(tmp_path) else str(bad) for x in base]
    r = subprocess.run([sys.executable] + tr + ["--master-port", str(_port())] + base_bad
                       + ["--resume"], cwd=ROOT, capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode != 0 and "inconsistent resume" in r.stderr
    other = [x if x != "5" else "6" for x in base]
    r = subprocess.run([sys.executable] + tr + ["--master-port", str(_port())] + other
                       + ["--resume"], cwd=ROOT, capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode != 0 and "same input on all ranks=False" in r.stderr


def test_als_script():
    out = _run(["matrix_computation/matrix_decomposition.py", "--device", "cpu"])
    assert out.count("rmse:") == 5 and "iterations: 4, rmse:" in out


def test_monte_carlo_script():
    out = _run(["randomized_algorithm/monte_carlo.py", "--device", "cpu"])
    assert "Pi is roughly 3.1" in out


def test_torchrun_two_ranks_gloo():
    out = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                "optimization/bmuf.py", "--device", "cpu", "--backend", "gloo",
                "--n-iterations", "20", "--quiet", "--no-plot"], timeout=400)
    assert out.count("Final acc:") == 1   # rank 0 prints only


def test_torchrun_hung_rank_fails_fast():
    """A rank that stops making progress ends a 2-rank gloo entry-script run non-zero
    within the deadlines (process-group timeout on the waiting rank, stall watchdog on
    the hung one) instead of hanging until torchrun is killed."""
    import time
    env = dict(os.environ, PYTHONPATH=ROOT, DALGO_TEST_HANG="1:fit")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), "optimization/ssgd.py", "--device", "cpu",
                        "--backend", "gloo", "--n-iterations", "20", "--quiet", "--no-plot",
                        "--pg-timeout-s", "10", "--stall-timeout-s", "15"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    el = time.time() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    assert el < 120, el
    assert "DALGO_TEST_HANG at fit" in r.stderr


def test_checkpoint_resume(tmp_path):
    ck = str(tmp_path / "ck")
    full = _run(["optimization/easgd.py", "--device", "cpu", "--n-iterations", "40", "--quiet",
                 "--no-plot"])
    _run(["optimization/easgd.py", "--device", "cpu", "--n-iterations", "20", "--quiet",
          "--no-plot", "--ckpt-dir", ck])
    resumed = _run(["optimization/easgd.py", "--device", "cpu", "--n-iterations", "40", "--quiet",
                    "--no-plot", "--ckpt-dir", ck, "--resume"])
    assert "Resumed from iteration 20" in resumed
    fw = full.split("Final w:")[1]
    rw = resumed.split("Final w:")[1]
    assert fw == rw


@pytest.mark.parametrize("script,args,final", [
    ("machine_learning/k-means.py", ["--synthetic", "3000,4", "--k", "5", "--n-iterations", "6"],
     "Final centers:"),
    ("graph_computation/pagerank.py", ["--rmat-scale", "9", "--top", "5", "--n-iterations", "6"],
     "has rank:"),
    ("matrix_computation/matrix_decomposition.py", ["--n-iterations", "6"], "iterations: 5, rmse:"),
])
def test_checkpoint_resume_other_apps(tmp_path, script, args, final):
    """Run 6 iterations straight vs. 3 + resume to 6: identical final output."""
    ck = str(tmp_path / "ck")
    base = [script, "--device", "cpu", "--no-plot"]
    full = _run(base + args)
    short = [x if x != "6" else "3" for x in args]
    _run(base + short + ["--ckpt-dir", ck])
    resumed = _run(base + args + ["--ckpt-dir", ck, "--resume"])
    assert "Resumed from iteration 3" in resumed
    tail = lambda out: out[out.index(final):]
    assert tail(full) == tail(resumed)


def test_bench_cpu_contract():
    out = _run(["bench.py", "--device", "cpu", "--rows", "20000", "--dim", "64", "--steps", "3",
                "--warmup", "1", "--dtype", "f32"])
    line = [l for l in out.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0


def test_bench_self_launches_n_ranks():
    """python bench.py --gpus 2 with no launcher environment starts 2 ranks itself
    (torchrun child process) and reports dp2 with both ranks' device records."""
    out = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--backend", "gloo", "--rows", "20000",
                "--dim", "64", "--steps", "3", "--warmup", "1", "--dtype", "f32", "--n-test", "5000"],
               timeout=600)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["config"]["parallelism"] == "dp2"
    assert len(d["device_ids"]) == 2 and d["allreduce_us_per_step"] > 0
    assert d["correctness_witness"]["passed"] and d["correctness_witness"]["trained_steps"] == 1500


@pytest.mark.parametrize("script,args,metric", [
    ("bench/kmeans_bench.py", ["--rows", "20000", "--dim", "16", "--k", "8", "--dtype", "f32",
                               "--iters", "2"], "k-means points/sec (whole node)"),
    ("bench/pagerank_bench.py", ["--scale", "10", "--steps", "2"], "PageRank edges/sec (whole node)"),
])
def test_secondary_benches_self_launch(script, args, metric):
    """The k-means and PageRank benches start N ranks themselves like bench.py."""
    out = _run([script, "--gpus", "2", "--device", "cpu", "--backend", "gloo"] + args, timeout=600)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["metric"] == metric and d["n_gpus"] == 2 and d["value"] > 0


def test_bench_refuses_mismatched_world():
    """--gpus N under a launcher with WORLD_SIZE != N fails loudly (no silent 1-GPU number)."""
    env = dict(os.environ, PYTHONPATH=ROOT, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--rows",
                        "2000", "--dim", "16", "--steps", "1", "--warmup", "0"], cwd=ROOT,
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stdout + r.stderr)


def test_module_dispatcher():
    """python -m dalgo <algorithm>: every reference script is reachable by name."""
    out = _run(["-m", "dalgo", "list"])
    for name in ("ssgd", "ma", "bmuf", "easgd", "logistic_regression", "kmeans", "pagerank",
                 "transitive_closure", "als", "monte_carlo"):
        assert name in out
    out = _run(["-m", "dalgo", "pagerank", "--device", "cpu", "--no-plot"])
    assert "1 has rank: 0.38891305880091237." in out
    out = _run(["-m", "dalgo", "closure", "--device", "cpu"])
    assert "The original graph has 9 paths" in out
    r = subprocess.run([sys.executable, "-m", "dalgo", "nope"], cwd=ROOT, capture_output=True,
                       text=True, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 2


def _top_ranks(out):
    res = {}
    for line in out.splitlines():
        if " has rank: " in line:
            v, r = line.split(" has rank: ")
            res[int(v)] = float(r.rstrip("."))
    return res


def test_pagerank_rmat_world_size_invariant():
    """R-MAT PageRank with the degree relabeling (dealt over the W slices): 1 rank and 3
    gloo ranks report the same top vertices (generator ids) and ranks."""
    args = ["graph_computation/pagerank.py", "--device", "cpu", "--rmat-scale", "10",
            "--top", "10"]
    one = _top_ranks(_run(args))
    three = _top_ranks(_run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                             "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
                            + ["--backend", "gloo"], timeout=400))
    assert len(one) == 10 and set(one) == set(three)
    assert max(abs(one[v] - three[v]) for v in one) < 1e-12
    # 3 ranks take the overlapped ghost exchange by default (own-source share 1/3); the
    # sequential exchange + single SpMV pass gives the same ranks
    seq = _top_ranks(_run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
                          + ["--backend", "gloo", "--overlap", "off"], timeout=400))
    assert set(seq) == set(three) and max(abs(seq[v] - three[v]) for v in seq) < 1e-12


def test_metrics_jsonl_phases_two_ranks(tmp_path):
    """--metrics-out: one JSONL line per iteration with the phase split and the bytes
    all-reduced (2 gloo ranks: non-zero bytes)."""
    m = tmp_path / "m.jsonl"
    _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
          "--master-addr", "127.0.0.1", "--master-port", str(_port()),
          "optimization/ssgd.py", "--device", "cpu", "--backend", "gloo", "--n-iterations", "6",
          "--quiet", "--no-plot", "--metrics-out", str(m)], timeout=400)
    recs = [json.loads(l) for l in m.read_text().splitlines()]
    assert [r["iteration"] for r in recs] == list(range(1, 7))
    assert set(recs[0]["phase_ms"]) >= {"sample+grad", "allreduce", "update", "eval"}
    assert recs[-1]["bytes_allreduced"] == 6 * 32 * 8 and recs[0]["world_size"] == 2
    m2 = tmp_path / "k.jsonl"
    _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
          "--master-addr", "127.0.0.1", "--master-port", str(_port()),
          "machine_learning/k-means.py", "--device", "cpu", "--backend", "gloo",
          "--synthetic", "2000,8", "--k", "4", "--no-plot", "--metrics-out", str(m2)], timeout=400)
    recs = [json.loads(l) for l in m2.read_text().splitlines()]
    assert len(recs) == 5 and set(recs[0]["phase_ms"]) >= {"assign", "accumulate", "allreduce",
                                                           "update"}
    assert recs[-1]["bytes_allreduced"] == 5 * 4 * (4 * 16 + 2 * 4)


def test_bench_recovers_from_device_wait_failure():
    """A device-side wait failure reported by one rank after the timed region: every rank
    falls back to the plain per-step form, re-runs warmup + timed steps and the bench
    still reports a valid (witness-checked) number, flagged in the JSON."""
    out = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--backend", "gloo", "--rows", "20000",
                "--dim", "64", "--steps", "3", "--warmup", "1", "--dtype", "f32", "--n-test", "5000"],
               env_extra={"DALGO_TEST_FORCE_DEVICE_ERROR": "1"}, timeout=600)
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["device_wait_fallback"] is True and d["n_gpus"] == 2
    assert d["correctness_witness"]["passed"]
    # the hook also left partial sums (1e3) in the gradient bucket, as a launch that
    # stopped early would: the fallback must clear them, so the re-measured run equals a
    # clean run exactly (same sample count, same trained model)
    clean = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--backend", "gloo", "--rows",
                  "20000", "--dim", "64", "--steps", "3", "--warmup", "1", "--dtype", "f32",
                  "--n-test", "5000"], timeout=600)
    c = json.loads([l for l in clean.splitlines() if l.startswith("{")][0])
    assert c["device_wait_fallback"] is False
    assert d["config"]["global_batch"] == c["config"]["global_batch"]
    assert d["correctness_witness"]["heldout_logloss"] == c["correctness_witness"]["heldout_logloss"]


def test_bench_local_sgd_counts_exact():
    """MA / BMUF / EASGD report the device-counted sample total (every local model's
    minibatch at every local step), not an estimate from rows * frac: it equals the exact
    Bernoulli selection of the timed steps (same Philox stream as the kernels)."""
    import numpy as np
    from dalgo.utils.philox import bernoulli_mask
    rows, warm, steps = 4000, 1, 3
    for algo, n_local in (("bmuf", 5), ("easgd", 1)):
        out = _run(["bench.py", "--device", "cpu", "--rows", str(rows), "--dim", "16", "--steps",
                    str(steps), "--warmup", str(warm), "--dtype", "f32", "--n-test", "1000",
                    "--algo", algo, "--no-eval"], timeout=600)
        d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
        idx = np.arange(rows, dtype=np.uint64)
        exp = n_local * sum(int(bernoulli_mask(42, t, idx, 0.1).sum())
                            for t in range(warm, warm + steps))
        assert d["samples_counted"] == exp, (algo, d["samples_counted"], exp)
