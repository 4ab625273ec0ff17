#!/usr/bin/env python3
"""Headline benchmark: whole-job tokens/s of Llama-3-8B CLM pre-training (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI between them). Every step is a full training step of the real
Llama-3-8B architecture (h 4096, I 14336, 32 layers, 32 q / 8 kv heads, vocab 128256, random init,
bf16 weights + fp32 master/Adam state): forward, backward, gradient reduction, norm clipping (1.0)
and the fused AdamW update. Data is synthetic: four sequences of S=8192 random tokens per GPU per
step (micro-batch 4 by default: 260 GiB peak of the 268 GiB HBM at dp=1, weak scaling). W untimed warm-up steps, then exactly K timed steps between
a barrier + device synchronize on both sides; the reported time is the MAX over ranks. Rank 0
prints one JSON line.

Other BASELINE.json configs (``--workload``; same JSON schema, their own metric string):
  pt-packed  Llama-3-8B CLM with ``--packed-docs K`` isolated documents per row (varlen attention)
  it         Phi-3-mini instruction tuning, NEFTune (alpha 5), GROUP_BY_LENGTH-style packed rows of
             4096 tokens with segment ids (no cross-contamination), loss on ~half the tokens
  dpo / orpo Llama-3-8B preference tuning: chosen + rejected sequences of 4096 tokens each per
             micro-batch (DPO adds the frozen reference model's forward)
  gpt2-cpu   GPT-2 small CLM on the CPU, one process (plumbing; config #1, no GPU needed)
TP / SP: ``--tp 2`` (the driver's scaling runs use the default data-parallel layout).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

LLAMA3_8B = dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                 num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192, rope_theta=500000.0,
                 rms_norm_eps=1e-5, bos_token_id=128000, eos_token_id=128001, tie_word_embeddings=False)
# Phi-3-mini-128k-instruct geometry (LongRoPE tables with neutral factors: the HF factor lists are not
# available offline; they do not change the compute)
PHI3_MINI = dict(vocab_size=32064, hidden_size=3072, intermediate_size=8192, num_hidden_layers=32,
                 num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=131072,
                 original_max_position_embeddings=4096, rope_theta=10000.0, rms_norm_eps=1e-5,
                 rope_scaling={"type": "longrope", "short_factor": [1.0] * 48, "long_factor": [1.0] * 48},
                 bos_token_id=1, eos_token_id=32000, pad_token_id=32000)

# workload -> (metric, model name, default seq len, default micro-batch)
WORKLOADS = {
    "pt": ("tokens/sec (whole node) Llama-3-8B CLM pre-train", "Llama-3-8B", 8192, 4),
    # per-GPU micro-batches sized for 288 GB of HBM (peak 264 / 253 GiB): pt-packed 4 x 8192 as pt; Phi-3 IT
    # 16 x 4096 (50.2k tok/s vs 49.6k at 12 and 49.3k at 8 on one box: the optimizer and the per-step fixed
    # costs spread over twice the tokens)
    "pt-packed": ("tokens/sec (whole node) Llama-3-8B CLM pre-train, isolated packed documents", "Llama-3-8B",
                  8192, 4),
    "it": ("tokens/sec (whole node) Phi-3-mini instruction tuning, NEFTune + varlen packing", "Phi-3-mini-128k",
           4096, 16),
    # DPO / ORPO: pairs per micro-batch (x 2 sides x 4096 tokens); DPO 3 (244 GiB, its frozen reference
    # model adds 16 GB), ORPO 4
    "dpo": ("tokens/sec (whole node) Llama-3-8B DPO preference tuning", "Llama-3-8B", 4096, 3),
    "orpo": ("tokens/sec (whole node) Llama-3-8B ORPO preference tuning", "Llama-3-8B", 4096, 4),
    "gpt2-cpu": ("tokens/sec GPT-2 small CLM pre-train on CPU (plumbing)", "GPT-2-small", 1024, 2),
}
# GPT-2 small (124 M) through HFCausalLM: BASELINE.json config #1, a CPU plumbing run
GPT2_SMALL = dict(model_type="gpt2", n_layer=12, n_head=12, n_embd=768, vocab_size=50257, n_positions=1024)


def bench_gpt2_cpu(args):
    """One process, no GPU: the whole stack (HF model wrapper, fused-loss CLM head, flat-buffer engine
    with AdamW, clipping) on the CPU torch reference ops. Not a performance number."""
    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.hf_causal_lm import HFCausalLM, HFCausalLMConfig
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    metric, model_name, S_def, mb_def = WORKLOADS["gpt2-cpu"]
    S, B = args.seq or S_def, args.micro_batch or mb_def
    torch.manual_seed(1234)
    model = HFCausalLM(HFCausalLMConfig(hf_config=dict(GPT2_SMALL), loss_chunk_size=args.loss_chunk))
    model.init_weights(1234)
    engine = DataParallelEngine(model, ParallelContext.single(), 0, lr=3e-4, weight_decay=0.1)
    lm = CLM({"model": None})
    lm.model = model
    lm.train()
    g = torch.Generator().manual_seed(1000)
    batches = [torch.randint(0, GPT2_SMALL["vocab_size"], (B, S), generator=g) for _ in range(args.warmup + args.steps)]

    def step(ids):
        engine.begin_step(1)
        engine.zero_grad()
        engine.begin_micro(0)
        loss, _, _ = lm.training_step({"input_ids": ids, "labels": ids})
        loss.backward()
        engine.finish_backward()
        engine.clip_and_scale(1.0)
        engine.step(3e-4)
        return loss

    for i in range(args.warmup):
        step(batches[i])
    t0 = time.perf_counter()
    losses = [float(step(batches[args.warmup + i]).detach()) for i in range(args.steps)]
    el = time.perf_counter() - t0
    tps = B * S * args.steps / el
    print(json.dumps({
        "metric": metric, "value": round(tps, 2), "unit": "tokens/s", "n_gpus": 0, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1000, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (random tokens, random-init weights)",
        "config": {"model": model_name, "global_batch": B, "seq_len": S, "parallelism": "cpu-1proc",
                   "zero_stage": 0, "optimizer": "AdamW fp32 (torch reference ops)", "grad_clip": 1.0,
                   "workload": "gpt2-cpu", "torch_threads": torch.get_num_threads()},
        "final_loss": round(losses[-1], 4), "losses": [round(x, 4) for x in losses]}), flush=True)


def flops_per_token(cfg: dict, S: int, attn_frac: float = 1.0) -> float:
    """6 x matmul params + causal attention FLOPs per token (attn_frac < 1 for packed documents)."""
    h, I, L, V = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"], cfg["vocab_size"]
    hq, hkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    d = h // hq
    n_matmul = L * (h * (hq + 2 * hkv) * d + hq * d * h + 3 * h * I) + V * h
    attn = L * 6 * 2 * S * h / 2 * attn_frac  # causal: 6 (fwd+bwd) x 2 matmuls x S x h x 1/2
    return 6 * n_matmul + attn


def doc_lengths(S: int, n: int, g: torch.Generator) -> list[int]:
    """n random document lengths summing to S (best-fit-packed rows hold a few documents each)."""
    cuts = sorted(torch.randint(1, S, (n - 1,), generator=g).tolist()) if n > 1 else []
    edges = [0, *cuts, S]
    return [b - a for a, b in zip(edges[:-1], edges[1:]) if b > a]


def probe_collectives(pc, device, mb: float, iters: int = 5) -> dict:
    """Bus bandwidth (GB/s) of an all-gather and a reduce-scatter of ``mb`` MB of bf16 over the data-parallel
    group (the world when dp is 1: TP collectives then), the engine's per-unit collectives. busbw =
    bytes of the full buffer / time x (n - 1) / n, the usual ring-normalised figure: one xGMI link direction
    (~153 GB/s on a full-mesh MI355X node) bounds a ring."""
    group = pc.dp_group if pc.dp_size > 1 else None
    n = pc.dp_size if pc.dp_size > 1 else dist.get_world_size()
    numel = int(mb * 1e6 / 2) // (n * 64) * (n * 64)
    full = torch.empty(numel, dtype=torch.bfloat16, device=device)
    part = torch.ones(numel // n, dtype=torch.bfloat16, device=device)
    out = {"probe_group": n, "probe_mb": round(numel * 2 / 1e6, 1)}
    for name, fn in (("ag", lambda: dist.all_gather_into_tensor(full, part, group=group)),
                     ("rs", lambda: dist.reduce_scatter_tensor(part, full, group=group))):
        fn()
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        sec = a.elapsed_time(b) / 1e3 / iters
        t = torch.tensor([sec], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sec = float(t.item())
        out[f"{name}_ms"] = round(sec * 1e3, 3)
        out[f"{name}_busbw_gbs"] = round(numel * 2 / sec * (n - 1) / n / 1e9, 1)
    del full, part
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="pt", choices=sorted(WORKLOADS))
    ap.add_argument("--seq", type=int, default=None, help="sequence length (per side for dpo/orpo)")
    ap.add_argument("--micro-batch", type=int, default=None)
    ap.add_argument("--packed-docs", type=int, default=8, help="pt-packed / it: documents per row")
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer layers (result marked invalid)")
    ap.add_argument("--zero-stage", type=int, default=None)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--attn", default="flash", choices=["flash", "sdpa", "eager"])
    ap.add_argument("--impl", default="native", choices=["native", "hf"],
                    help="pt / pt-packed: the native Llama, or transformers' LlamaForCausalLM through HFCausalLM "
                         "(HIP attention, fused RMSNorm / SwiGLU patch, fused loss head)")
    ap.add_argument("--ckpt", action="store_true", help="full activation checkpointing")
    ap.add_argument("--ckpt-keep-attn", action="store_true",
                    help="with --ckpt: keep the flash-attention outputs (recompute_granularity full_keep_attention)")
    ap.add_argument("--offload-optimizer", action="store_true", help="fp32 master/Adam state in host memory")
    ap.add_argument("--loss-chunk", type=int, default=8192, help="rows per lm_head GEMM of the fused CE")
    ap.add_argument("--force-sharded", action="store_true",
                    help="run the dp>1 engine schedule (RCCL reduce-scatter/all-gather, comm stream) even on 1 GPU")
    ap.add_argument("--gemm-tuning", default=None, choices=["use", "tune", "off"],
                    help="hipBLASLt solution selection (default: shipped TunableOp results)")
    ap.add_argument("--step-timeout", type=float, default=180.0,
                    help="watchdog: seconds one step (or the collective probe) may take before every rank dumps "
                         "its stacks and the job exits non-zero (0: off)")
    ap.add_argument("--setup-timeout", type=float, default=420.0,
                    help="watchdog limit for process-group setup, model build and the first step")
    ap.add_argument("--probe-mb", type=float, default=436.0,
                    help="size of the untimed all-gather / reduce-scatter bandwidth probe (one Llama-3-8B layer "
                         "unit in bf16); 0: skip")
    args = ap.parse_args()
    if args.workload == "gpt2-cpu":
        bench_gpt2_cpu(args)
        return
    # `python bench.py --gpus N` without torchrun: start N rank processes here (no HIP call in this
    # parent) and exit with the job's code; under torchrun / srun WORLD_SIZE must equal --gpus
    from llm_training_amd.launch import maybe_launch
    rc = maybe_launch(args.gpus, [sys.executable, os.path.abspath(__file__), *sys.argv[1:]])
    if rc is not None:
        sys.exit(rc)

    from llm_training_amd.ops.native import lib
    from llm_training_amd.parallel.context import ParallelContext, init_distributed
    from llm_training_amd.parallel.engine import DataParallelEngine
    from llm_training_amd.runtime.gemm_tuning import setup_gemm_tuning
    from llm_training_amd.runtime.monitor import StepWatchdog

    metric, model_name, S_def, mb_def = WORKLOADS[args.workload]
    S = args.seq or S_def
    B = args.micro_batch or mb_def
    wd = StepWatchdog(int(os.environ.get("RANK", "0")), args.step_timeout)
    wd.arm("process-group setup and model build", args.setup_timeout if args.step_timeout > 0 else 0)
    rank, local, world, device = init_distributed()
    if args.force_sharded and world == 1:
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=device)
    gemm_mode = setup_gemm_tuning(args.gemm_tuning)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    comm_backend = None
    if dist.is_initialized():
        # the multi-GPU run must really be one RCCL communicator over every GPU (torch's "nccl" backend is
        # RCCL on ROCm); LLMT_DIST_BACKEND=gloo is the test knob for several ranks on one GPU
        comm_backend = dist.get_backend()
        want = os.environ.get("LLMT_DIST_BACKEND") or "nccl"
        if comm_backend != want or dist.get_world_size() != args.gpus:
            raise SystemExit(f"expected a {want} process group of {args.gpus} ranks, got {comm_backend} "
                             f"with {dist.get_world_size()}")
    lib()  # fail loudly if the HIP extension is missing
    pc = ParallelContext.create("auto", args.tp, device)

    phi3 = args.workload == "it"
    cfg = dict(PHI3_MINI if phi3 else LLAMA3_8B)
    if args.layers:
        cfg["num_hidden_layers"] = args.layers
    common = dict(attn_implementation=args.attn, enable_gradient_checkpointing=args.ckpt,
                  loss_chunk_size=args.loss_chunk)
    if args.ckpt and args.ckpt_keep_attn:
        common["recompute_granularity"] = "full_keep_attention"
    if phi3:
        from llm_training_amd.models.phi3 import Phi3 as Model
        from llm_training_amd.models.phi3 import Phi3Config as MCfg
    else:
        from llm_training_amd.models.llama import Llama as Model
        from llm_training_amd.models.llama import LlamaConfig as MCfg
    if args.impl == "hf":
        if phi3 or args.workload in ("dpo", "orpo") or args.tp > 1:
            raise SystemExit("--impl hf: the pt / pt-packed workloads without tensor parallelism")
        from llm_training_amd.models.hf_causal_lm import HFCausalLM as Model
        from llm_training_amd.models.hf_causal_lm import HFCausalLMConfig
        hf = {k: v for k, v in cfg.items()}
        hf.update(model_type="llama", torch_dtype="bfloat16")
        mcfg = HFCausalLMConfig(hf_config=hf, attn_implementation=args.attn, enable_liger_kernel=True,
                                enable_gradient_checkpointing=args.ckpt, loss_chunk_size=args.loss_chunk)
    else:
        mcfg = MCfg(**cfg, **common)
    torch.manual_seed(1234)
    model = Model(mcfg, pc, dtype=torch.bfloat16, device=device)
    model.init_weights(seed=1234)
    stage = args.zero_stage if args.zero_stage is not None else (0 if pc.dp_size == 1 else 2)
    engine = DataParallelEngine(model, pc, stage, lr=3e-5, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1,
                                offload_optimizer=args.offload_optimizer, force_sharded=args.force_sharded)
    if args.workload in ("dpo", "orpo"):
        from llm_training_amd.lms.preference import DPO, ORPO
        lm = (DPO if args.workload == "dpo" else ORPO)({"model": None, "beta": 0.1})
        lm.model = model
        if args.workload == "dpo":
            ref = Model(mcfg, pc, dtype=torch.bfloat16, device=device)
            ref.load_state_dict(model.state_dict())
            ref.requires_grad_(False)
            ref.eval()
            lm.ref_model = ref
    else:
        from llm_training_amd.lms.clm import CLM
        lm = CLM({"model": None, "neftune_alpha": 5.0 if phi3 else None})
        lm.model = model
    lm.train()

    V = cfg["vocab_size"]
    g = torch.Generator(device=device).manual_seed(1000 + pc.dp_rank)
    gcpu = torch.Generator().manual_seed(2000 + pc.dp_rank)
    attn_work = []  # fraction of full-causal attention work per step (packed documents)

    def packed_segments(n_docs):
        seg = torch.empty(B, S, dtype=torch.int32)
        frac = 0.0
        for b in range(B):
            lens = doc_lengths(S, n_docs, gcpu)
            seg[b] = torch.repeat_interleave(torch.arange(1, len(lens) + 1, dtype=torch.int32), torch.tensor(lens))
            frac += sum(ln * ln for ln in lens) / (S * S)
        attn_work.append(frac / B)
        return seg.to(device)

    def make_batch():
        if args.workload in ("dpo", "orpo"):
            out = {}
            for side in ("chosen", "rejected"):
                ids = torch.randint(0, V, (B, S), device=device, generator=g)
                lab = ids.clone()
                lab[:, : S // 4] = -100  # the prompt part carries no loss
                out.update({f"{side}_input_ids": ids, f"{side}_labels": lab,
                            f"{side}_attention_mask": torch.ones(B, S, dtype=torch.long, device=device)})
            attn_work.append(1.0)
            return out
        ids = torch.randint(0, V, (B, S), device=device, generator=g)
        batch = {"input_ids": ids, "labels": ids, "position_ids": torch.arange(S, device=device).expand(B, S),
                 "attention_mask": None}
        if args.workload in ("pt-packed", "it"):
            batch["attention_mask"] = packed_segments(args.packed_docs)
            batch["attention_mask_trivial"] = False
            if args.workload == "it":  # loss only on the "assistant" part of the documents
                lab = ids.clone()
                lab[torch.rand(B, S, device=device, generator=g) < 0.5] = -100
                batch["labels"] = lab
        else:
            attn_work.append(1.0)
        return batch

    hang = os.environ.get("LLMT_BENCH_HANG")  # test knob "rank:step": that rank stops at that step
    hang_rank, hang_step = (int(x) for x in hang.split(":")) if hang else (-1, -1)
    n_step = [0]

    def step(batch):
        if rank == hang_rank and n_step[0] == hang_step:
            print(f"[rank {rank}] LLMT_BENCH_HANG: stopping at step {hang_step}", file=sys.stderr, flush=True)
            while True:
                time.sleep(1.0)
        n_step[0] += 1
        engine.begin_step(1)
        engine.zero_grad()
        engine.begin_micro(0)
        loss, _, _ = lm.training_step(batch)
        loss.backward()
        engine.finish_backward()
        engine.clip_and_scale(1.0)
        engine.step(3e-5)
        return loss

    # untimed: bandwidth of one layer-unit all-gather / reduce-scatter over the data-parallel group
    rccl = {"backend": comm_backend, "world": world}
    # the collective-library knobs this run saw (RCCL / NCCL channel, protocol, MSCCL settings): set by the
    # user or launcher, never hard-coded here, and recorded with the numbers they produced
    knobs = {k: v for k, v in sorted(os.environ.items()) if k.startswith(("NCCL_", "RCCL_"))}
    if knobs:
        rccl["env"] = knobs
    if dist.is_initialized() and args.probe_mb > 0:
        wd.arm("collective bandwidth probe")
        rccl.update(probe_collectives(pc, device, args.probe_mb))

    # fresh synthetic batches for every step (pre-generated so the timed loop does no data work)
    batches = [make_batch() for _ in range(args.warmup + args.steps)]
    # the host runs at most one step ahead of the device (it waits for step i-1's event after queueing
    # step i, so the device never idles): a step that hangs on the device trips the watchdog within
    # --step-timeout of its start instead of at the final synchronize
    prev = [None]

    def run(i, label, limit=None):
        wd.arm(label, limit)
        out = step(batches[i])
        ev = torch.cuda.Event()
        ev.record()
        if prev[0] is not None:
            prev[0].synchronize()
        prev[0] = ev
        return out

    for i in range(args.warmup):
        loss = run(i, f"warm-up step {i}", args.setup_timeout if i == 0 and args.step_timeout > 0 else None)
    wd.arm("synchronize before the timed steps")
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    prev[0] = None
    meter = {}
    engine.wait_meter = meter
    from llm_training_amd.parallel import tensor_parallel as tpl
    if pc.tp_size > 1:  # compute-stream stalls on the staged TP collectives (tensor_parallel._tp_wait)
        tpl.TP_WAIT_METER = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = run(args.warmup + i, f"timed step {i}", args.setup_timeout if args.warmup == 0 and i == 0
                   and args.step_timeout > 0 else None)
    wd.arm("synchronize after the timed steps")
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    el_host = time.perf_counter() - t0
    engine.wait_meter = None
    waits = engine.wait_meter_ms(meter)
    rccl["exposed_comm_ms_per_step"] = round(waits.get("comm", 0.0) / args.steps, 3)
    rccl["exposed_optimizer_wait_ms_per_step"] = round(waits.get("opt", 0.0) / args.steps, 3)
    if tpl.TP_WAIT_METER is not None:
        rccl["exposed_tp_comm_ms_per_step"] = round(
            sum(a.elapsed_time(b) for a, b in tpl.TP_WAIT_METER) / args.steps, 3)
        # the chunk count actually used for this shard (tp_stages reduces LLMT_TP_STAGES to divide the shard)
        # and the chunks per GEMM of every staged projection
        rccl["tp_stages"] = tpl.tp_stages(S // pc.tp_size)
        rccl["tp_gemm_groups"] = dict(tpl.STAGE_PLANS)
        tpl.TP_WAIT_METER = None
    el = torch.tensor([el_host], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.item()
    final_loss = float(loss.detach().float().item())
    seqs = 2 * B if args.workload in ("dpo", "orpo") else B
    tokens = pc.dp_size * seqs * S * args.steps
    tps = tokens / el
    timed = attn_work[args.warmup:]
    frac = sum(timed) / max(1, len(timed))
    fpt = flops_per_token(cfg, S, frac)
    if args.workload == "dpo":
        fpt += flops_per_token(cfg, S, frac) / 3  # frozen reference model: forward only
    peak_mem = torch.cuda.max_memory_allocated(device) / 2 ** 30
    import llm_training_amd.ops.fused as F_layouts
    from llm_training_amd.ops.native import llmt_env
    if rank == 0:
        par = f"dp{pc.dp_size}" + (f"-tp{pc.tp_size}" if pc.tp_size > 1 else "")
        cfg_out = {"model": model_name if not args.layers else f"{model_name}-{args.layers}L(INVALID-debug)",
                   "global_batch": pc.dp_size * B, "seq_len": S, "parallelism": par, "zero_stage": stage,
                   "attn": args.attn,
                   "activation_checkpointing": ("full_keep_attention" if args.ckpt and args.ckpt_keep_attn
                                                else args.ckpt),
                   "optimizer": ("host AdamW (offload) fp32 master" if args.offload_optimizer
                                 else "fused AdamW fp32 master"),
                   "grad_clip": 1.0, "gemm_tuning": gemm_mode}
        if args.workload != "pt":
            cfg_out["workload"] = args.workload
        if args.impl != "native":
            cfg_out["impl"] = "transformers LlamaForCausalLM (HFCausalLM, fused-kernel patch)"
        if args.workload in ("pt-packed", "it"):
            cfg_out.update(packed_docs_per_row=args.packed_docs, attn_work_vs_causal=round(frac, 4))
        if phi3:
            cfg_out["neftune_alpha"] = 5.0
        # the schedule actually run: one GPU defaults to ZeRO-0 (no collectives); several GPUs to ZeRO-2
        # (the reference example's DeepSpeed stage); force_sharded runs the dp>1 schedule on one GPU
        cfg_out["force_sharded"] = bool(args.force_sharded)
        if stage == 2 and pc.dp_size > 1:
            # the FSDP schedule it matches: parameters gathered once per step (FSDP2
            # reshard_after_forward=False), gradients reduce-scattered, optimizer state sharded
            cfg_out["fsdp_equivalent"] = "FSDP2 reshard_after_forward=False"
        out = {
            "metric": metric,
            "value": round(tps, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1000, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)", "config": cfg_out,
            "tokens_per_sec_per_gpu": round(tps / world, 2),
            "mfu": round(tps / world * fpt / 2.5e15, 4),
            "tflops_per_gpu": round(tps / world * fpt / 1e12, 1),
            "peak_mem_gib": round(peak_mem, 1),
            "final_loss": round(final_loss, 4),
            "rccl": rccl,
            # how the GEMM layouts were chosen (shipped table / timed / rank 0's) and the hash of the choices
            "gemm_layouts": F_layouts.layout_summary(),
            # every LLMT_* knob of the environment (kernel variants, layouts, schedules) this number ran with
            "llmt_env": llmt_env(),
        }
        if os.environ.get("LLMT_GEMM_LAYOUT_DUMP"):
            F_layouts.dump_layouts(os.environ["LLMT_GEMM_LAYOUT_DUMP"])
        if os.environ.get("LLMT_GEMM_LT_EXPORT"):  # hipBLASLt's solution per problem ("key rank ms name gsuN")
            from llm_training_amd.ops.native import lib as _lib
            with open(os.environ["LLMT_GEMM_LT_EXPORT"], "w") as f:
                f.write(_lib().gemm_lt_export())
        print(json.dumps(out), flush=True)
    wd.arm("shutdown")
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    wd.disarm()


if __name__ == "__main__":
    main()
