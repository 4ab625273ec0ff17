"""The tensor-parallel autograd functions on the GPU over a one-rank RCCL group: the overlapped
all-gather + GEMM (`_AGLinear`), GEMM + reduce-scatter (`_LinearRS`) and the vocab-parallel loss heads
(`_VPFusedCE`, `_VPLogps`) run their RCCL calls and native GEMM / CE paths (at tp = 1 the public
wrappers short-circuit to the plain ops, so these are called directly) and must match fp32 torch."""
import pytest
import torch
import torch.distributed as dist

from llm_training_amd.ops import reference as ref
from llm_training_amd.parallel import tensor_parallel as tpl
from llm_training_amd.parallel import vocab_parallel as vp
from tests.helpers import free_port

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def group():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                                device_id=dev)
        created = True
    yield dist.group.WORLD
    if created:
        dist.destroy_process_group()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("fn", ["ag", "rs"])
def test_overlapped_tp_linears(group, fn):
    torch.manual_seed(0)
    S, B, K, N = 256, 2, 512, 768
    x = torch.randn(S, B, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (0.05 * torch.randn(N, K, device="cuda")).bfloat16().requires_grad_(True)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    f = tpl._AGLinear if fn == "ag" else tpl._LinearRS
    y = f.apply(x, w, b, group)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr.t() + br
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    assert _rel(b.grad, br.grad) < 1e-2


@pytest.mark.parametrize("head", ["ce", "logps", "logps-recompute"])
def test_vocab_parallel_heads(group, head):
    torch.manual_seed(0)
    N, H, V = 1024, 256, 5000
    h = torch.randn(N, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (0.05 * torch.randn(V, H, device="cuda")).bfloat16().requires_grad_(True)
    lab = torch.randint(0, V, (N,), device="cuda")
    lab[::7] = -100
    hr, wr = h.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    if head == "ce":
        out = vp._VPFusedCE.apply(h, w, lab, 0, -100, group, 256, V)
        out.backward()
        torch.nn.functional.cross_entropy(hr @ wr.t(), lab, ignore_index=-100).backward()
        assert abs(out.item() - torch.nn.functional.cross_entropy(hr @ wr.t(), lab).item()) < 2e-2
    else:
        keep = 0 if head == "logps-recompute" else 1 << 40  # logits recomputed in backward / kept
        out, rs = vp._VPLogps.apply(h, w, lab, 0, -100, group, 256, V, keep)
        assert _rel(rs, (hr @ wr.t()).sum(-1)) < 1e-2  # logit row sums (ORPO metrics)
        gg = torch.randn_like(out)
        (out * gg).sum().backward()
        lr_ = ref.token_logps(hr @ wr.t(), lab)
        (lr_ * gg).sum().backward()
        assert _rel(out, lr_) < 1e-2
    assert _rel(h.grad, hr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2
