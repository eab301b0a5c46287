"""Native LSD radix sort (csrc/kernels/radix_sort.hip) behind the adjacency build's sorts:
stable sort on a bit range == torch's stable sort of the same field, for tile-ragged sizes,
skewed (one hot digit) and uniform keys; the look-back error word stays clear."""
import os
import subprocess
import sys

import pytest
import torch

from dalgo.ops import _ext

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the sort backend is chosen once per process (DALGO_SORT): the native sort is checked in
# a child process with DALGO_SORT=native, the default (rocPRIM) one here


def _field(x, lo, hi):
    return (x >> lo) & ((1 << (hi - lo)) - 1) if hi < 63 else x >> lo


@pytest.mark.parametrize("n,lo,hi", [(1, 0, 8), (4095, 0, 16), (4097, 3, 40), (1_000_003, 12, 52),
                                     (3_000_001, 0, 63), (300_000, 20, 27)])
def test_native_sort_matches_stable_torch(cuda, n, lo, hi):
    g = torch.Generator().manual_seed(n)
    keys = torch.randint(0, 1 << 62, (n,), generator=g, dtype=torch.int64)
    keys[: n // 3] &= ~(((1 << 8) - 1) << lo)          # a third share one digit per pass (hot)
    keys = keys.to(cuda)
    out = torch.empty_like(keys)
    ops = _ext.ops()
    ops.gb_sort(keys, n, hi, out, lo)
    f = _field(keys.cpu(), lo, hi)
    exp = keys.cpu()[torch.sort(f, stable=True).indices]
    assert torch.equal(out.cpu(), exp)
    assert int(ops.rs_sort_error(keys).item()) == 0


def test_native_sort_partial_prefix(cuda):
    """Sorting keys[:n] of a longer buffer leaves out[n:] alone."""
    keys = torch.randint(0, 1 << 40, (50_000,), device=cuda)
    out = torch.full_like(keys, -5)
    _ext.ops().gb_sort(keys, 40_000, 40, out, 0)
    assert torch.equal(out[:40_000].cpu(), torch.sort(keys[:40_000].cpu()).values)
    assert bool((out[40_000:] == -5).all())


def test_native_sort_in_child_process(cuda):
    """The same checks with DALGO_SORT=native (the native reduce-then-scan radix sort)."""
    env = dict(os.environ, DALGO_SORT="native", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", __file__,
                        "-k", "not child_process", "-p", "no:cacheprovider"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed" in r.stdout
