"""The multi-GPU engine schedule on ONE GPU: ``force_sharded`` runs every dp > 1 code path (comm stream,
events, RCCL reduce-scatter / all-gather over a one-rank group, stage-3 free / regather / prefetch,
transient stage >= 2 gradient buffers, offload copies) and must train exactly like the plain stage-0
engine. With deterministic kernels and a one-rank group (a reduce-scatter is a copy) the losses and
weights are bitwise identical at one micro-batch per step."""
import os

import pytest
import torch
import torch.distributed as dist

from llm_training_amd.lms.clm import CLM
from llm_training_amd.models.llama import Llama, LlamaConfig
from llm_training_amd.parallel.context import ParallelContext
from llm_training_amd.parallel.engine import DataParallelEngine
from tests.helpers import free_port

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_group():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                                device_id=dev)
        created = True
    yield dev
    if created:
        dist.destroy_process_group()


def _cfg(**kw):
    base = dict(vocab_size=4096, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=2048, rope_theta=500000.0)
    base.update(kw)
    return LlamaConfig(**base)


def _run(dev, stage, forced, ckpt=False, accum=1, offload=False, steps=3, S=512, **eng_kw):
    torch.manual_seed(0)
    cfg = _cfg(enable_gradient_checkpointing=ckpt)
    m = Llama(cfg, ParallelContext.single(dev), dtype=torch.bfloat16, device=dev)
    m.init_weights(5)
    eng = DataParallelEngine(m, ParallelContext.single(dev), stage, lr=1e-3, force_sharded=forced,
                             offload_optimizer=offload, **eng_kw)
    lm = CLM({"model": None})
    lm.model = m
    lm.train()
    g = torch.Generator(device=dev).manual_seed(11)
    losses = []
    peak_transient = 0
    for _ in range(steps):
        eng.begin_step(accum)
        eng.zero_grad()
        tot = 0.0
        for i in range(accum):
            eng.begin_micro(i)
            ids = torch.randint(0, cfg.vocab_size, (1, S), device=dev, generator=g)
            loss, _, _ = lm.training_step({"input_ids": ids, "labels": ids})
            loss.backward()
            peak_transient = max(peak_transient, eng.grad_memory_bytes()["transient"])
            tot += loss.item() / accum
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-3)
        losses.append(tot)
    with eng.full_params_context():
        eng.wait_params()
        params = {k: v.float().cpu() for k, v in m.state_dict().items()}
    torch.cuda.synchronize()
    return losses, params, eng, peak_transient


@pytest.mark.parametrize("stage,ckpt", [(1, False), (2, False), (2, True), (3, False), (3, True)])
def test_forced_sharded_matches_stage0_bitwise(rccl_group, monkeypatch, stage, ckpt):
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")
    dev = rccl_group
    ref_l, ref_p, _, _ = _run(dev, 0, forced=False)
    l, p, eng, peak = _run(dev, stage, forced=True, ckpt=ckpt)
    assert eng.sharded and eng.comm_stream is not None
    assert l == ref_l, (l, ref_l)
    bad = [k for k in ref_p if not torch.equal(p[k], ref_p[k])]
    assert not bad, bad
    if stage >= 2:
        # transient layer gradients are gone after every backward (reduce-scattered, then freed)
        assert peak == 0
        assert sum(u.transient_grad for u in eng.units) == 3


@pytest.mark.parametrize("stage", [2, 3])
def test_forced_sharded_accumulation_matches_stage0(rccl_group, monkeypatch, stage):
    """Two micro-batches per step: stage >= 2 reduce-scatters every micro-batch and accumulates the
    shards (bf16 adds in another order than the stage-0 in-place GEMM accumulation)."""
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")
    dev = rccl_group
    ref_l, ref_p, _, _ = _run(dev, 0, forced=False, accum=2)
    l, p, _, _ = _run(dev, stage, forced=True, ckpt=True, accum=2)
    for a, b in zip(l, ref_l):
        assert abs(a - b) < 1e-3 * abs(b), (l, ref_l)
    num = den = 0.0
    for k in ref_p:
        num += (p[k] - ref_p[k]).norm().item() ** 2
        den += ref_p[k].norm().item() ** 2
    assert (num / den) ** 0.5 < 2e-3


def test_forced_sharded_offload_matches_device(rccl_group, monkeypatch):
    """Stage 2 + optimizer offload on the sharded path (D2H of reduced shards on the copy stream, host
    AdamW, H2D + all-gather) vs the device AdamW on the same path."""
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")
    dev = rccl_group
    ref_l, ref_p, _, _ = _run(dev, 2, forced=True)
    l, p, eng, _ = _run(dev, 2, forced=True, offload=True)
    assert eng.units[1].master.device.type == "cpu"
    for a, b in zip(l, ref_l):
        assert abs(a - b) < 2e-4 * abs(b), (l, ref_l)
    num = den = 0.0
    for k in ref_p:
        num += (p[k] - ref_p[k]).norm().item() ** 2
        den += ref_p[k].norm().item() ** 2
    assert (num / den) ** 0.5 < 3e-3  # host vs device AdamW rounding (measured 1.1e-3)


def test_checkpoint_save_resume_sharded_offload(rccl_group, tmp_path, monkeypatch):
    """Save on the sharded + offload path (host-resident optimizer shards, no collective needed), load
    into a fresh engine, and continue: identical next-step loss to an uninterrupted run."""
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")
    from llm_training_amd.ckpt.checkpoint import load_checkpoint, save_checkpoint

    dev = rccl_group

    class _T:  # the slice of Trainer that save/load use
        pass

    def make(offload):
        torch.manual_seed(0)
        m = Llama(_cfg(), ParallelContext.single(dev), dtype=torch.bfloat16, device=dev)
        m.init_weights(5)
        eng = DataParallelEngine(m, ParallelContext.single(dev), 2, lr=1e-3, force_sharded=True,
                                 offload_optimizer=offload)
        lm = CLM({"model": None})
        lm.model = m
        from llm_training_amd.runtime.trainer import TrainerState
        t = _T()
        t.pc, t.engine, t.lm, t.state, t.scheduler, t.config_dict = (ParallelContext.single(dev), eng, lm,
                                                                     TrainerState(), None, None)
        return t

    def step(t, ids):
        e = t.engine
        e.begin_step(1)
        e.zero_grad()
        e.begin_micro(0)
        loss, _, _ = t.lm.training_step({"input_ids": ids, "labels": ids})
        loss.backward()
        e.finish_backward()
        e.clip_and_scale(1.0)
        e.step(1e-3)
        return loss.item()

    g = torch.Generator(device=dev).manual_seed(3)
    batches = [torch.randint(0, 4096, (1, 256), device=dev, generator=g) for _ in range(3)]
    a = make(True)
    step(a, batches[0])
    step(a, batches[1])
    save_checkpoint(a, str(tmp_path / "ck"))
    want = step(a, batches[2])
    b = make(True)
    load_checkpoint(b, str(tmp_path / "ck"))
    assert b.engine.step_count == 2
    got = step(b, batches[2])
    assert got == want, (got, want)


@pytest.mark.parametrize("offload,kw,exact", [
    (False, {"offload_params": True}, True),
    (True, {"offload_params": True}, False),
    (False, {"quantized_weights": True}, True),  # one rank: its own exact slice is the whole unit
    (False, {"quantized_gradients": True}, False),
])
def test_forced_sharded_zero3_offload_and_zeropp(rccl_group, monkeypatch, offload, kw, exact):
    """Stage 3 with parameter offload (pinned host shards, H2D into the gather buffer on the comm
    stream), and the int8 ZeRO++ paths (csrc/quant.hip + RCCL all-gather / all-to-all)."""
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")
    dev = rccl_group
    ref_l, ref_p, _, _ = _run(dev, 0, forced=False)
    l, p, eng, _ = _run(dev, 3 if "quantized_gradients" not in kw else 2, forced=True, offload=offload, **kw)
    if kw.get("offload_params"):
        assert eng.units[1].pshard.device.type == "cpu" and eng.units[1].pshard.is_pinned()
    if exact:
        assert l == ref_l, (l, ref_l)
        assert all(torch.equal(p[k], ref_p[k]) for k in ref_p)
    else:
        for a, b in zip(l, ref_l):
            assert abs(a - b) < 1e-2 * abs(b), (l, ref_l)


@pytest.mark.parametrize("stage,forced,packed", [(0, False, False), (2, True, False), (3, True, True)])
def test_training_step_has_no_host_sync(rccl_group, stage, forced, packed):
    """a steady-state training step (forward, fused loss, backward, reduce-scatter /
    all-gather, clipping, fused AdamW) never blocks the host on the GPU. torch's sync debug mode turns
    any implicit synchronisation (a D2H copy, .item(), a blocking allocator retry, nonzero) into an
    error; the batch (incl. packed segment ids and the collator's ``attention_mask_trivial`` flag) is
    built before the window, as the data loader does."""
    dev = rccl_group
    torch.manual_seed(0)
    cfg = _cfg()
    m = Llama(cfg, ParallelContext.single(dev), dtype=torch.bfloat16, device=dev)
    m.init_weights(5)
    eng = DataParallelEngine(m, ParallelContext.single(dev), stage, lr=1e-3, force_sharded=forced)
    lm = CLM({"model": None})
    lm.model = m
    lm.train()
    S = 512
    ids = torch.randint(0, cfg.vocab_size, (2, S), device=dev)
    batch = {"input_ids": ids, "labels": ids}
    if packed:
        seg = torch.repeat_interleave(torch.tensor([1, 2, 3]), torch.tensor([200, 100, 212]))
        batch.update(attention_mask=seg.expand(2, S).to(dev), attention_mask_trivial=False,
                     position_ids=torch.cat([torch.arange(200), torch.arange(100), torch.arange(212)])
                     .expand(2, S).to(dev))

    def step():
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(batch)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-3)
        return loss

    step()  # warm-up: allocator pools, GEMM solution lookup, ring buffers
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        loss = step()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()


def test_generic_optimizer_on_the_sharded_gpu_path(rccl_group, monkeypatch):
    """A generic torch optimizer (SGD with momentum) on the optimizer stream over the fp32 master pieces:
    forced ZeRO-2 == plain stage 0, bitwise (deterministic kernels, one-rank reduce-scatter = copy)."""
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")
    import functools
    dev = rccl_group
    fac = functools.partial(torch.optim.SGD, lr=1e-2, momentum=0.9)
    ref_l, ref_p, e0, _ = _run(dev, 0, forced=False, optimizer_factory=fac)
    l, p, e2, _ = _run(dev, 2, forced=True, optimizer_factory=fac)
    assert type(e2.units[1].opt).__name__ == "SGD" and e2.units[1].opt.state
    assert l == ref_l, (l, ref_l)
    assert all(torch.equal(p[k], ref_p[k]) for k in ref_p)
    assert l[-1] < l[0]


def test_dpo_reference_model_gather_only_on_gpu(rccl_group):
    """The ZeRO-3 gather-only reference model on the GPU path (comm-stream all-gathers into the
    ring, prefetch, release): its log-probs equal the unsharded reference's."""
    from llm_training_amd.lms.preference import DPO
    from llm_training_amd.parallel.frozen import FrozenShards
    dev = rccl_group
    lm = DPO({"model": {"model_class": "llm_training.models.Llama",
                        "model_config": dict(vocab_size=4096, hidden_size=512, intermediate_size=1024,
                                             num_hidden_layers=3, num_attention_heads=8, num_key_value_heads=2)}})
    lm.configure_model(ParallelContext.single(dev), dev, torch.bfloat16, seed=3)
    g = torch.Generator(device=dev).manual_seed(1)
    b = {}
    for side in ("chosen", "rejected"):
        ids = torch.randint(0, 4096, (2, 256), device=dev, generator=g)
        b.update({f"{side}_input_ids": ids, f"{side}_labels": ids,
                  f"{side}_attention_mask": torch.ones_like(ids)})
    with torch.no_grad():
        want = lm.logps(lm.ref_model, b)
    fs = FrozenShards(lm.ref_model, dist.group.WORLD, 0, 1, torch.cuda.Stream(device=dev))
    for _ in range(2):
        with torch.no_grad():
            got = lm.logps(lm.ref_model, b)
        fs.release_all()
        assert all(torch.equal(x, y) for x, y in zip(got, want))
    assert sum(p.numel() for p in lm.ref_model.parameters()) == 0  # nothing bound between forwards
