"""Metrics parity (reference src/llm_training/metrics/*): counts, perplexity, in-place state load, DP reduction."""
import math

import torch

from llm_training_amd.metrics import ConsumedSamples, ConsumedTokens, Perplexity
from tests.helpers import run_gloo


def test_consumed_counters_and_state_roundtrip():
    cs, ct = ConsumedSamples(), ConsumedTokens(ignore_index=-100)
    t = torch.tensor([[1, 2, -100], [4, -100, -100]])
    cs.update(t)
    ct.update(t)
    cs.update(t)
    ct.update(t)
    assert cs.compute().item() == 4 and ct.compute().item() == 6
    sd = ct.state_dict()
    ct2 = ConsumedTokens()
    ref = ct2.n
    ct2.load_state_dict(sd)
    assert ct2.compute().item() == 6 and ct2.n is ref  # copied in place


def test_perplexity_scalar_and_token_level():
    p = Perplexity()
    p.update(torch.tensor(2.0))
    p.update(torch.tensor(4.0))
    assert abs(p.compute().item() - math.exp(3.0)) < 1e-4
    torch.manual_seed(0)
    logits = torch.randn(2, 5, 11)
    tgt = torch.randint(0, 11, (2, 5))
    tgt[0, 0] = -100
    q = Perplexity(ignore_index=-100)
    q.update(logits, tgt)
    nll = torch.nn.functional.cross_entropy(logits.reshape(-1, 11), tgt.reshape(-1), ignore_index=-100)
    assert abs(q.compute().item() - math.exp(nll.item())) < 1e-4
    q.reset()
    assert q.count.item() == 0


def _dist_worker(rank, world):
    cs = ConsumedSamples()
    cs.update(torch.zeros(rank + 1, 3))
    pp = Perplexity()
    pp.update(torch.tensor(float(rank)))
    return {"n": cs.compute().item(), "ppl": pp.compute().item()}


def test_metrics_reduce_over_data_parallel_group():
    out = run_gloo(_dist_worker, 2)
    for r in (0, 1):
        assert out[r]["n"] == 3
        assert abs(out[r]["ppl"] - math.exp(0.5)) < 1e-5


def test_utils_parity():
    import contextlib

    import torch.nn as nn

    from llm_training_amd.models.utils import init_empty_weights, init_on_device
    from llm_training_amd.utils import ContextManagers, StrEnum, copy_method_signature

    order = []

    @contextlib.contextmanager
    def cm(i):
        order.append(("in", i))
        yield
        order.append(("out", i))

    with ContextManagers([cm(1), cm(2)]):
        pass
    assert order == [("in", 1), ("in", 2), ("out", 2), ("out", 1)]

    class Color(StrEnum):
        RED = __import__("enum").auto()
        BLUE = "Blue"

    assert Color.RED == "red" and str(Color.BLUE) == "Blue"

    class A:
        def f(self, x: int, y: int = 2):
            """doc"""
            return x + y

    class B(A):
        @copy_method_signature(A.f)
        def f(self):
            ...

    assert B().f(1) == 3 and "y" in str(__import__("inspect").signature(B.f))
    with init_empty_weights():
        lin = nn.Linear(4, 4)
    assert lin.weight.device.type == "meta"
    with init_on_device("cpu", include_buffers=True):
        lin2 = nn.Linear(2, 2)
    assert lin2.weight.device.type == "cpu"


def test_slurm_nodelist_first_host():
    from llm_training_amd.parallel.context import first_slurm_host
    assert first_slurm_host("gpu[03-05,9],cpu1") == "gpu03"
    assert first_slurm_host("nodeA,nodeB") == "nodeA"
    assert first_slurm_host("mi355x-017") == "mi355x-017"
    assert first_slurm_host("") is None
