"""Tensor-parallel random streams (gloo, CPU ranks): every TP rank of a DP group draws its own dropout
masks / NEFTune noise / attention-dropout seeds (they act on different head or sequence shards), while
the data-parallel layout keeps seed + dp_rank."""
import torch

from tests.helpers import run_gloo


def _rng_worker(rank, world, tp):
    from llm_training_amd.data.dummy import DummyDataModule
    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.ops import fused as F_
    from llm_training_amd.ops import reference as ref
    from llm_training_amd.runtime.strategies import FSDP2Strategy
    from llm_training_amd.runtime.trainer import Trainer
    lm = CLM({"model": {"model_class": "llm_training.models.Llama",
                        "model_config": {"vocab_size": 96, "hidden_size": 32, "intermediate_size": 64,
                                         "num_hidden_layers": 1, "num_attention_heads": 4,
                                         "num_key_value_heads": 2, "attention_dropout": 0.5}},
              "optim": {"optimizer_class": "torch.optim.AdamW", "optimizer_kwargs": {"lr": 1e-2}}})
    dm = DummyDataModule({"batch_size": 2, "vocab_size": 96, "max_length": 16, "num_samples": 16, "base_seed": 5})
    t = Trainer(strategy=FSDP2Strategy(tensor_parallel_size=tp), precision="32-true", max_steps=1, seed=3)
    t.setup(lm, dm)
    seed = F_.dropout_seed()
    # the same local head's attention with dropout on identical inputs: the mask is this rank's
    g = torch.Generator().manual_seed(0)
    q = torch.randn(1, 16, 2, 8, generator=g)
    o = ref.attention_dropout(q, q, q, True, None, -1, 0.35, 0.5, seed)
    return {"tp_rank": t.pc.tp_rank, "dp_rank": t.pc.dp_rank, "seed": seed, "o": o, "noise": torch.rand(8)}


def test_tp_ranks_draw_distinct_dropout_streams():
    res = run_gloo(_rng_worker, 4, (2,))  # dp2 x tp2
    res = [res[r] for r in sorted(res)]
    by = {(r["dp_rank"], r["tp_rank"]): r for r in res}
    for d in range(2):
        a, b = by[(d, 0)], by[(d, 1)]
        assert a["seed"] != b["seed"]
        assert not torch.equal(a["o"], b["o"])  # same local head, same inputs, different masks
        assert not torch.equal(a["noise"], b["noise"])
    # and every (dp, tp) stream is distinct
    assert len({r["seed"] for r in res}) == 4


def _it_batches(n, B=2, S=15, V=128, seed=0):
    """Instruction-tuning-like packed rows of odd length: segment ids, loss on part of the tokens."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(1, V, (B, S), generator=g)
        seg = torch.ones(B, S, dtype=torch.long)
        seg[:, 6:] = 2
        seg[1, 11:] = 0  # trailing padding of row 1
        lab = ids.clone()
        lab[torch.rand(B, S, generator=g) < 0.4] = -100
        lab[seg == 0] = -100
        out.append({"input_ids": ids, "labels": lab, "attention_mask": seg, "attention_mask_trivial": False})
    return out


def _tp_it_worker(rank, world, tp, full0, batches, neftune):
    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    from tests.helpers import tiny_llama_cfg
    pc = ParallelContext.create("auto", tp, "cpu") if tp > 1 else ParallelContext.single()
    m = Llama(tiny_llama_cfg(), pc, dtype=torch.float32)
    m.load_full_state_dict(full0)
    eng = DataParallelEngine(m, pc, 2 if pc.dp_size > 1 else 0, lr=1e-2, weight_decay=0.0)
    lm = CLM({"model": None, "neftune_alpha": neftune})
    lm.model = m
    lm.train()
    losses = []
    for b in batches:
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(b)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-2)
        losses.append(loss.item())
    with eng.full_params_context():
        sd = m.gather_full_state_dict() if pc.tp else {k: v.detach().clone() for k, v in m.state_dict().items()}
    return {"losses": losses, "params": sd}


def test_tp2_odd_sequence_length_matches_single_process():
    """S = 15 at TP = 2: right-padded to 16 inside the model, stripped again; losses and weights equal
    the single-process run (reference DTensor Shard(1) handles uneven shards)."""
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from tests.helpers import tiny_llama_cfg
    m = Llama(tiny_llama_cfg(), ParallelContext.single(), dtype=torch.float32)
    m.init_weights(1)
    full0 = {k: v.clone() for k, v in m.state_dict().items()}
    batches = _it_batches(3)
    ref = run_gloo(_tp_it_worker, 1, (1, full0, batches, None))[0]
    out = run_gloo(_tp_it_worker, 2, (2, full0, batches, None))
    for r in (0, 1):
        for a, b in zip(out[r]["losses"], ref["losses"]):
            assert abs(a - b) < 1e-5, (out[r]["losses"], ref["losses"])
        for k, v in ref["params"].items():
            # the staged TP GEMMs sum the weight gradient in (stage, rank) blocks: fp32 rounding of a
            # different summation order, which Adam's g / sqrt(v) at lr 1e-2 amplifies to ~3e-5 on a few
            # elements (of 16k) after three steps
            assert torch.allclose(out[r]["params"][k], v, atol=1e-4, rtol=1e-4), k


def test_tp2_odd_length_with_neftune_runs():
    """NEFTune's per-token noise mask is padded with the sequence (no shape error on the last shard)."""
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from tests.helpers import tiny_llama_cfg
    m = Llama(tiny_llama_cfg(), ParallelContext.single(), dtype=torch.float32)
    m.init_weights(1)
    full0 = {k: v.clone() for k, v in m.state_dict().items()}
    out = run_gloo(_tp_it_worker, 2, (2, full0, _it_batches(2), 5.0))
    assert all(x == x for x in out[0]["losses"])
