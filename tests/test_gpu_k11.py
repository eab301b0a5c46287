"""K11 (csrc/kernels/xgmi_allreduce.hip) at world = 1, in the default GPU tier: the
exchange kernel, its device-resident epoch walk (both buffer phases over back-to-back
calls), and the fused SSGD / GD update tail against the separate K8 (sync_update).
One rank pushes into its own slot and waits on its own flag: no cross-process wait,
so this is safe on a single GPU (the multi-rank K11 rehearsals are the opt-in
``gpu_shared`` set). It replaces the treeAggregate of optimization/ssgd.py:99-103."""
import pytest
import torch

from dalgo.ops import _ext
from dalgo.ops.update import GD_SUM, SSGD, sync_update

pytestmark = pytest.mark.gpu


class _OneRank:
    def __init__(self, cuda, slot=4096):
        self.ops = _ext.ops()
        self.slot = slot
        self.own = int(self.ops.xgmi_alloc(int(self.ops.xgmi_buffer_bytes(slot)), cuda.index or 0))
        self.epoch = torch.zeros(1, dtype=torch.int32, device=cuda)
        self.err = torch.zeros(1, dtype=torch.int32, device=cuda)

    def __call__(self, x, **upd):
        if upd:
            self.ops.xgmi_allreduce(x, [self.own], 0, self.slot, self.epoch, self.err, 2.0,
                                    upd["W"], upd["mode"], 0, upd["eta"], 0.0, 0.0,
                                    upd["count_index"], upd.get("count_acc"))
        else:
            self.ops.xgmi_allreduce(x, [self.own], 0, self.slot, self.epoch, self.err, 2.0)
        return x

    def close(self):
        torch.cuda.synchronize()
        self.ops.xgmi_free(self.own)


def test_k11_one_rank_plain_sum(cuda):
    k11 = _OneRank(cuda)
    try:
        for it in range(6):                      # both buffer phases, epoch advancing
            n = 1031 + 517 * it
            ref = torch.randn(n, device=cuda)
            x = ref.clone()
            k11(x)
            torch.cuda.synchronize()
            assert torch.equal(x, ref), it
        assert int(k11.epoch.item()) != 0
        assert int(k11.err.item()) == 0
    finally:
        k11.close()


@pytest.mark.parametrize("mode", [SSGD, GD_SUM])
def test_k11_one_rank_fused_update_matches_sync_update(cuda, mode):
    """[g || count] through K11 with the fused update == sync_update on the same bucket;
    the fused form leaves the bucket zeroed and accumulates the sample count."""
    D = 1025
    g = torch.Generator(device="cpu").manual_seed(3)
    k11 = _OneRank(cuda)
    try:
        W0 = torch.randn(D, generator=g).to(cuda)
        W_f, W_r = W0.clone(), W0.clone()
        acc = torch.zeros(1, dtype=torch.float64, device=cuda)
        for step in range(4):
            grad = torch.randn(D, generator=g).to(cuda)
            cnt = float(100 + step)
            x = torch.cat([grad, torch.tensor([cnt], device=cuda)])
            xr = x.clone()
            k11(x, W=W_f, mode=mode, eta=0.1, count_index=D, count_acc=acc)
            sync_update(W_r, mode, G=xr[:D], C=xr[D:], eta=0.1)
            torch.cuda.synchronize()
            assert torch.allclose(W_f, W_r, rtol=1e-6, atol=1e-7), (step, (W_f - W_r).abs().max())
            assert not bool(x.abs().sum().item()), "bucket must be left zeroed"
        assert float(acc.item()) == sum(100 + s for s in range(4))
        assert int(k11.err.item()) == 0
    finally:
        k11.close()
