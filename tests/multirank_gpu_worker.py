"""Rank process for tests/test_multirank_gpu.py: two ranks share cuda:0 over the gloo backend (RCCL
refuses two ranks on one GPU), so the dp_rank > 0 / tp_rank > 0 code paths of the engine, TP+SP and the
loss heads run with the real HIP kernels and real cross-rank data. Writes rank 0's losses and full
parameters to ``OUT``."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dpo_main(out):
    """DPO at dp2 x ZeRO-3 with the gather-only dp-sharded reference model (parallel/frozen.py)."""
    from llm_training_amd.lms.preference import DPO
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    from tests.multirank_gpu_common import CFG, pref_batches
    dev = torch.device("cuda", 0)
    pc = ParallelContext.create("auto", 1, dev)
    lm = DPO({"model": {"model_class": "llm_training.models.Llama", "model_config": CFG.model_dump()}, "beta": 0.1})
    lm.configure_model(pc, dev, torch.bfloat16, seed=5)
    eng = DataParallelEngine(lm.model, pc, 3, lr=1e-3, weight_decay=0.0)
    lm.on_engine_ready(eng)
    assert lm.ref_shards is not None
    lm.train()
    losses = []
    for b in pref_batches(dev):
        B = b["chosen_input_ids"].shape[0] // pc.dp_size
        local = {k: v[pc.dp_rank * B:(pc.dp_rank + 1) * B] for k, v in b.items()}
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(local)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-3)
        t = loss.detach().float().reshape(1)
        dist.all_reduce(t)
        losses.append(t.item() / dist.get_world_size())
    held = sum(p.numel() for p in lm.ref_model.parameters())
    with eng.full_params_context():
        eng.wait_params()
        sd = {k: v.detach().float().cpu() for k, v in lm.model.state_dict().items()}
    torch.cuda.synchronize()
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "params": sd, "ref_held": held,
                    "ref_shard_bytes": lm.ref_shards.resident_bytes()}, out)
    dist.barrier()


def main():
    mode, out = sys.argv[1], sys.argv[2]  # mode: dp2_z2 | dp2_z3 | tp2 | dpo_z3
    dist.init_process_group("gloo")
    if mode == "dpo_z3":
        dpo_main(out)
        dist.destroy_process_group()
        return
    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    from tests.multirank_gpu_common import CFG, STEPS, batches
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tp = 2 if mode == "tp2" else 1
    stage = {"dp2_z2": 2, "dp2_z3": 3, "tp2": 0}[mode]
    pc = ParallelContext.create("auto", tp, dev)
    m = Llama(CFG, pc, dtype=torch.bfloat16, device=dev)
    full0 = torch.load(os.environ["FULL0"], weights_only=True)
    m.load_full_state_dict({k: v.to(dev) for k, v in full0.items()})
    eng = DataParallelEngine(m, pc, stage, lr=1e-3, weight_decay=0.0)
    lm = CLM({"model": None})
    lm.model = m
    lm.train()
    losses = []
    for ids in batches(dev):
        B = ids.shape[0] // pc.dp_size
        local = ids[pc.dp_rank * B:(pc.dp_rank + 1) * B]
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step({"input_ids": local, "labels": local})
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-3)
        t = loss.detach().float().reshape(1)
        dist.all_reduce(t)
        losses.append(t.item() / dist.get_world_size())
    with eng.full_params_context():
        eng.wait_params()
        sd = m.gather_full_state_dict() if pc.tp else {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    torch.cuda.synchronize()
    # every rank's hipBLASLt solution per problem (key -> "rank gsuN"): rank 0's after agree_layouts
    from llm_training_amd.ops.native import lib
    mine = {ln.split()[0]: ln.split()[1] + " " + ln.split()[-1] for ln in lib().gemm_lt_export().splitlines()}
    every = [None] * dist.get_world_size()
    dist.all_gather_object(every, mine)
    if dist.get_rank() == 0:
        torch.save({"losses": losses, "params": {k: v.float().cpu() for k, v in sd.items()},
                    "grad_norm": float(eng.grad_norm), "lt_choices": every}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
