"""Numerics of the LR kernels (K1/K7/K10) and K8 against the torch fp32/fp64 reference."""
import numpy as np
import pytest
import torch

from dalgo.ops import lr as L
from dalgo.ops import update as U
from dalgo.ops.lr import pad_features

pytestmark = pytest.mark.gpu


def _data(n, D, dtype, seed=0, device=None):
    """Uniform(-1, 1) rows and 0/1 labels; device=...: generated there (the large cases:
    1.25M x 1024 on the host took ~5 s of the suite)."""
    g = torch.Generator(device=device or "cpu").manual_seed(seed)
    X = (torch.rand((n, D), generator=g, device=device) * 2 - 1).to(dtype)
    y = (torch.rand(n, generator=g, device=device) < 0.5).float()
    return X, y


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("D", [30, 256, 1000, 1024])
@pytest.mark.parametrize("frac", [0.1, 1.0])
def test_lr_grad_matches_reference(cuda, dtype, D, frac):
    n = 5000
    X, y = _data(n, D, dtype)
    Xc = pad_features(X)
    nseg = 3
    seg = torch.tensor([0, 1500, 3001, n], dtype=torch.int64)
    W = torch.randn(nseg, D + 1, generator=torch.Generator().manual_seed(1)) * 0.1
    kw = dict(D=D, has_bias=True, eps=1e-6, seed=42, step=7, frac=frac, row_offset=12345)
    G_ref, C_ref = L.lr_grad(Xc.float(), y, W.double(), seg, **kw)
    Gd, Cd = L.lr_grad(pad_features(X.to(cuda)), y.to(cuda), W.to(cuda), seg.to(cuda), **kw)
    torch.cuda.synchronize()
    assert torch.equal(Cd.cpu().double(), C_ref), (Cd, C_ref)
    err = (Gd.cpu().double() - G_ref).abs().max().item()
    scale = G_ref.abs().max().item() + 1e-6
    assert err / scale < 2e-5, (err, scale)


@pytest.mark.parametrize("fine", [0, 8])
@pytest.mark.parametrize("D", [256, 1024, 2048])
def test_lr_grad_shapes_and_claims(cuda, fine, D):
    """Both register layouts of the launch shape (two row sets below 4 column chunks per
    lane, one set at 2048 columns) and both in-block claim modes (whole 256-row groups
    only / fine 64-row quarters at the end) select the same rows and sum the same
    gradient as the CPU reference, over several segments."""
    n = 40_000
    X, y = _data(n, D, torch.bfloat16, seed=21)
    seg = torch.tensor([0, 13_331, n], dtype=torch.int64)
    W = torch.randn(2, D + 1, generator=torch.Generator().manual_seed(3)) * 0.05
    kw = dict(D=D, frac=0.1, step=5, seed=7)
    G_ref, C_ref = L.lr_grad(X, y, W.double(), seg, **kw)
    Gd, Cd = L.lr_grad(X.to(cuda), y.to(cuda), W.to(cuda), seg.to(cuda), fine_groups=fine, **kw)
    torch.cuda.synchronize()
    assert torch.equal(Cd.cpu().double(), C_ref), (fine, Cd, C_ref)
    rel = (Gd.cpu().double() - G_ref).abs().max() / G_ref.abs().max()
    assert rel < 1e-4, (fine, rel)


def test_lr_grad_single_segment_deterministic(cuda):
    X, y = _data(200_000, 1024, torch.bfloat16, seed=3, device=cuda)
    Xd, yd = X.to(cuda), y.to(cuda)
    W = torch.randn(1, 1025, generator=torch.Generator().manual_seed(2)).to(cuda) * 0.05
    seg = torch.tensor([0, X.shape[0]], dtype=torch.int64, device=cuda)
    outs = [L.lr_grad(Xd, yd, W, seg, D=1024, frac=0.1, step=3, deterministic=True)
            for _ in range(3)]
    for G, C in outs[1:]:
        assert torch.equal(G, outs[0][0]) and torch.equal(C, outs[0][1])
    # the default atomic epilogue agrees to f32 rounding (order of the block sums)
    Ga, Ca = L.lr_grad(Xd, yd, W, seg, D=1024, frac=0.1, step=3, deterministic=False)
    assert torch.equal(Ca, outs[0][1])
    assert ((Ga - outs[0][0]).abs().max() / outs[0][0].abs().max()).item() < 1e-5
    # g_is_zero=True accumulates into the given (zero) buffers without a memset
    G0 = torch.zeros_like(Ga)
    C0 = torch.zeros_like(Ca)
    L.lr_grad(Xd, yd, W, seg, D=1024, frac=0.1, step=3, G=G0, C=C0, g_is_zero=True)
    assert torch.equal(C0, Ca)
    assert ((G0 - Ga).abs().max() / Ga.abs().max()).item() < 1e-5
    G_ref, C_ref = L.lr_grad(X.cpu(), y.cpu(), W.cpu().double(), seg.cpu(), D=1024, frac=0.1, step=3)
    assert float(outs[0][1].item()) == float(C_ref.item())
    rel = (outs[0][0].cpu().double() - G_ref).abs().max() / G_ref.abs().max()
    assert rel < 1e-4


@pytest.mark.parametrize("align", [4, 260])
@pytest.mark.parametrize("mode", ["atomic", "deterministic"])
def test_lr_grad_static_range_alignment(cuda, monkeypatch, align, mode):
    """K1 with block ranges that are not multiples of 256 rows (RPB_ALIGN 4 / 260):
    partial 256-row groups at every block end, Philox quads straddling block
    boundaries, a row_offset that is not a multiple of 4, and the deterministic and
    atomic epilogues; exact counts and G vs the f64 CPU reference."""
    monkeypatch.setattr(L, "RPB_ALIGN", align)
    n, D = 300_001, 256
    X, y = _data(n, D, torch.bfloat16, seed=8)
    Xd, yd = X.to(cuda), y.to(cuda)
    seg = torch.tensor([0, 100_003, n], dtype=torch.int64)
    W = torch.randn(2, D + 1, generator=torch.Generator().manual_seed(6)) * 0.05
    for step in range(3):
        kw = dict(D=D, frac=0.1, step=step, seed=13, row_offset=6)
        G_ref, C_ref = L.lr_grad(X, y, W.double(), seg, **kw)
        Gd, Cd = L.lr_grad(Xd, yd, W.to(cuda), seg.to(cuda), deterministic=(mode == "deterministic"),
                           **kw)
        torch.cuda.synchronize()
        assert torch.equal(Cd.cpu().double(), C_ref), (step, Cd, C_ref)
        rel = (Gd.cpu().double() - G_ref).abs().max() / G_ref.abs().max()
        assert rel < 1e-4, (step, rel)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_lr_eval(cuda, dtype):
    X, y = _data(7777, 100, dtype, seed=5)
    w = torch.randn(101, generator=torch.Generator().manual_seed(9))
    c_ref, l_ref = L.lr_eval(pad_features(X).float(), y, w.double(), D=100)
    c, l = L.lr_eval(pad_features(X.to(cuda)), y.to(cuda), w.to(cuda), D=100)
    assert abs(int(c.item()) - int(c_ref.item())) <= 2   # sigma==0.5 ties may flip in f32
    assert abs(float(l.item()) - float(l_ref.item())) < 1e-3


@pytest.mark.parametrize("mode", range(7))
def test_sync_update_modes(cuda, mode):
    g = torch.Generator().manual_seed(mode)
    nrow = 1 if mode in (U.AVERAGE, U.BMUF, U.ELASTIC_CENTER) else 3
    n = 1025
    W = torch.randn(nrow, n, generator=g)
    G = torch.randn(nrow, n, generator=g)
    C = torch.tensor([5.0, 0.0, 17.0][:nrow])
    center = torch.randn(n, generator=g)
    S = torch.randn(n, generator=g)
    Dl = torch.randn(n, generator=g)
    kw = dict(reg="elastic_net", eta=0.1, lam=0.01, alpha=0.01, reg_alpha=0.3, mu=0.9,
              zeta=0.1, beta=0.04, inv_p=0.25)
    if mode == U.GD_SUM:
        kw.pop("lam")
    Wc, Dc = W.clone().double(), Dl.clone().double()
    U.sync_update(Wc, mode, G=G.double(), C=C.double(), center=center.double(), S=S.double(),
                  Dl=Dc, **kw)
    Wd, Dd = W.to(cuda), Dl.to(cuda)
    U.sync_update(Wd, mode, G=G.to(cuda), C=C.to(cuda), center=center.to(cuda), S=S.to(cuda),
                  Dl=Dd, **kw)
    assert torch.allclose(Wd.cpu().double(), Wc, rtol=1e-5, atol=1e-5)
    assert torch.allclose(Dd.cpu().double(), Dc, rtol=1e-5, atol=1e-5)
    # zero_grad: same update, and the gradient-consuming modes leave G / C zeroed
    Wz, Gz, Cz = W.to(cuda), G.to(cuda), C.to(cuda)
    U.sync_update(Wz, mode, G=Gz, C=Cz, center=center.to(cuda), S=S.to(cuda),
                  Dl=Dl.to(cuda), zero_grad=True, **kw)
    assert torch.equal(Wz, Wd)
    consumes = mode in (U.SSGD, U.GD_SUM, U.LOCAL_MEAN, U.LOCAL_ELASTIC)
    assert bool((Gz == 0).all()) == consumes and bool((Cz == 0).all()) == consumes


def test_rows_sum_broadcast(cuda):
    W = torch.randn(4, 1025)
    out = torch.zeros(1025)
    U.rows_sum(W, out)
    od = torch.zeros(1025, device=cuda)
    U.rows_sum(W.to(cuda), od)
    assert torch.allclose(od.cpu(), out, atol=1e-5)
    src = torch.randn(1025)
    Wd = W.to(cuda)
    U.rows_broadcast(Wd, src.to(cuda))
    assert torch.equal(Wd.cpu(), src.expand(4, -1))


@pytest.mark.parametrize("mode,reg,pool", [(0, 0, 0.0), (0, 3, 0.0), (1, 0, 0.0), (0, 0, 0.2)])
def test_lr_grad_fused_tail_single_rank(cuda, mode, reg, pool, monkeypatch):
    """One-launch step (gradient + update in the last block) == lr_grad + K8 (also with
    the cross-block row pool: exact minibatch counts)."""
    monkeypatch.setattr(L, "POOL_FRAC_ONE", pool)
    monkeypatch.setattr(L, "POOL_MIN_ROWS", 0)
    Xd, yd = _data(300_000, 1024, torch.bfloat16, seed=11, device=cuda)
    X = Xd
    seg = torch.tensor([0, X.shape[0]], dtype=torch.int64, device=cuda)
    w0 = torch.randn(1, 1025, generator=torch.Generator().manual_seed(4)).to(cuda) * 0.05
    kw = dict(D=1024, frac=0.1, eps=0.0, seed=42)
    upd = dict(eta=0.1, lam=0.01, reg_alpha=0.3)
    # reference: separate gradient + update launches
    w_ref = w0.clone()
    acc_ref = torch.zeros(1, dtype=torch.float64, device=cuda)
    for t in range(3):
        G, C = L.lr_grad(Xd, yd, w_ref, seg, step=t, **kw)
        U.sync_update(w_ref, U.SSGD if mode == 0 else U.GD_SUM, G=G, C=C, reg=reg,
                      count_acc=acc_ref, **upd)
    # fused tail
    w = w0.clone()
    G = torch.zeros(1, 1025, device=cuda)
    C = torch.zeros(1, device=cuda)
    acc = torch.zeros(1, dtype=torch.float64, device=cuda)
    for t in range(3):
        L.lr_grad(Xd, yd, w, seg, step=t, G=G, C=C, g_is_zero=(t > 0),
                  tail=dict(mode=mode, reg=reg, count_acc=acc, xg=None, **upd), **kw)
    torch.cuda.synchronize()
    assert float(acc.item()) == float(acc_ref.item())
    assert bool((G == 0).all()) and bool((C == 0).all())
    rel = ((w - w_ref).abs().max() / w_ref.abs().max()).item()
    assert rel < 1e-5, rel


@pytest.mark.parametrize("mode,reg,n,pool", [(0, 0, 300_000, 0.0), (0, 3, 1_250_000, 0.0), (1, 0, 40_000, 0.0),
                                             (0, 0, 1_250_001, 0.15), (1, 0, 300_002, 0.3)])
def test_lr_grad_persistent_steps(cuda, mode, reg, n, pool, monkeypatch):
    """Persistent launch (K steps in one cooperative grid, epoch-released W) == K
    separate gradient + update steps; the release counter ends at base + K. With a
    cross-block pool (the top rows claimed in 64-row units by whichever block runs out
    first) every row is still taken exactly once: the minibatch sizes match exactly."""
    monkeypatch.setattr(L, "POOL_FRAC", pool)
    monkeypatch.setattr(L, "POOL_MIN_ROWS", 0)
    Xd, yd = _data(n, 1024, torch.bfloat16, seed=12, device=cuda)
    seg = torch.tensor([0, n], dtype=torch.int64, device=cuda)
    w0 = torch.randn(1, 1025, generator=torch.Generator().manual_seed(5)).to(cuda) * 0.05
    kw = dict(D=1024, frac=0.1, eps=0.0, seed=42)
    # GD applies the gradient SUM: a small step keeps 14 steps from amplifying the
    # (order-dependent) f32 rounding of the atomic block sums
    upd = dict(eta=0.1 if mode == 0 else 1e-3, lam=0.01, reg_alpha=0.3)
    K = 7
    w_ref = w0.clone()
    acc_ref = torch.zeros(1, dtype=torch.float64, device=cuda)
    for t in range(2 * K):
        G, C = L.lr_grad(Xd, yd, w_ref, seg, step=t, **kw)
        U.sync_update(w_ref, U.SSGD if mode == 0 else U.GD_SUM, G=G, C=C, reg=reg,
                      count_acc=acc_ref, **upd)
    w = w0.clone()
    G = torch.zeros(1, 1025, device=cuda)
    C = torch.zeros(1, device=cuda)
    acc = torch.zeros(1, dtype=torch.float64, device=cuda)
    for r in range(2):   # two launches: the epoch base carries over
        L.lr_grad(Xd, yd, w, seg, step=r * K, G=G, C=C, g_is_zero=True,
                  tail=dict(mode=mode, reg=reg, count_acc=acc, xg=None, nsteps=K, **upd), **kw)
    torch.cuda.synchronize()
    L.check_persistent()
    assert float(acc.item()) == float(acc_ref.item())
    assert bool((G == 0).all()) and bool((C == 0).all())
    rel = ((w - w_ref).abs().max() / w_ref.abs().max()).item()
    assert rel < 1e-4, rel


@pytest.mark.parametrize("n", [300_001, 1_250_000])
def test_lr_grad_row_pool_plain_launch(cuda, n, monkeypatch):
    """A plain gradient launch with the cross-block row pool (the last block only re-arms
    the ticket and the pool counter) == the same launch without it: the same selected-row
    count (exact) and gradient sum over several steps."""
    Xd, yd = _data(n, 1024, torch.bfloat16, seed=13, device=cuda)
    seg = torch.tensor([0, n], dtype=torch.int64, device=cuda)
    w = torch.randn(1, 1025, generator=torch.Generator().manual_seed(6)).to(cuda) * 0.05
    kw = dict(D=1024, frac=0.1, eps=0.0, seed=42)
    for t in range(4):
        monkeypatch.setattr(L, "POOL_FRAC_ONE", 0.0)
        G0, C0 = L.lr_grad(Xd, yd, w, seg, step=t, **kw)
        monkeypatch.setattr(L, "POOL_FRAC_ONE", 0.2)
        monkeypatch.setattr(L, "POOL_MIN_ROWS", 0)
        G1, C1 = L.lr_grad(Xd, yd, w, seg, step=t, **kw)
        torch.cuda.synchronize()
        assert float(C1.item()) == float(C0.item())
        assert torch.allclose(G1, G0, rtol=1e-4, atol=1e-3)
    L.check_persistent()


@pytest.mark.gpu
def test_lr_reset_rearms_stale_counters(cuda, monkeypatch):
    """After a failed launch (simulated: ticket, pool and hand-off counters left part-way),
    reset_persistent_error re-arms them: the next pooled plain launch gives the same
    selected-row count and gradient as a launch without the pool."""
    n = 300_000
    Xd, yd = _data(n, 1024, torch.bfloat16, seed=17, device=cuda)
    seg = torch.tensor([0, n], dtype=torch.int64, device=cuda)
    w = torch.randn(1, 1025, generator=torch.Generator().manual_seed(8)).to(cuda) * 0.05
    kw = dict(D=1024, frac=0.1, eps=0.0, seed=42)
    monkeypatch.setattr(L, "POOL_FRAC_ONE", 0.0)
    G0, C0 = L.lr_grad(Xd, yd, w, seg, step=3, **kw)
    monkeypatch.setattr(L, "POOL_FRAC_ONE", 0.2)
    monkeypatch.setattr(L, "POOL_MIN_ROWS", 0)
    G1, C1 = L.lr_grad(Xd, yd, w, seg, step=3, **kw)      # creates the pooled workspace
    torch.cuda.synchronize()
    for ws in L._ws_cache.values():                       # what an aborted launch leaves
        ws.ticket.fill_(5)
        ws.pool.fill_(3)
        ws.epoch.fill_(7)
        ws.epochs = 9
    L.reset_persistent_error()
    for ws in L._ws_cache.values():
        assert int(ws.ticket.item()) == 0 and int(ws.pool.abs().sum().item()) == 0
        assert int(ws.epoch.item()) == 0 and ws.epochs == 0
    G2, C2 = L.lr_grad(Xd, yd, w, seg, step=3, **kw)
    torch.cuda.synchronize()
    assert float(C1.item()) == float(C0.item()) == float(C2.item())
    assert torch.allclose(G2, G0, rtol=1e-4, atol=1e-3)
    L.check_persistent()
