#!/usr/bin/env python3
"""Headline benchmark: whole-job tokens/s of Llama-3-8B CLM pre-training (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI between them). Every step is a full training step of the real
Llama-3-8B architecture (h 4096, I 14336, 32 layers, 32 q / 8 kv heads, vocab 128256, random init,
bf16 weights + fp32 master/Adam state): forward, backward, gradient reduction, norm clipping (1.0)
and the fused AdamW update. Data is synthetic: three packed sequences of S=8192 random tokens per GPU
per step (micro-batch 3 by default, weak scaling). W untimed warm-up steps, then exactly K timed steps between
a barrier + device synchronize on both sides; the reported time is the MAX over ranks. Rank 0
prints one JSON line.
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


def flops_per_token(cfg: dict, S: int) -> float:
    h, I, L, V = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"], cfg["vocab_size"]
    hq, hkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    d = h // hq
    n_matmul = L * (h * (hq + 2 * hkv) * d + hq * d * h + 3 * h * I) + V * h
    attn = L * 6 * 2 * S * h / 2  # causal: 6 (fwd+bwd) x 2 matmuls x S x h x 1/2
    return 6 * n_matmul + attn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--micro-batch", type=int, default=3)
    ap.add_argument("--layers", type=int, default=None, help="debug only: fewer layers (result marked invalid)")
    ap.add_argument("--zero-stage", type=int, default=None)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--attn", default="flash", choices=["flash", "sdpa", "eager"])
    ap.add_argument("--ckpt", action="store_true", help="full activation checkpointing")
    ap.add_argument("--offload-optimizer", action="store_true", help="fp32 master/Adam state in host memory")
    ap.add_argument("--loss-chunk", type=int, default=8192, help="rows per lm_head GEMM of the fused CE")
    ap.add_argument("--force-sharded", action="store_true",
                    help="run the dp>1 engine schedule (RCCL reduce-scatter/all-gather, comm stream) even on 1 GPU")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--gemm-tuning", default=None, choices=["use", "tune", "off"],
                    help="hipBLASLt solution selection (default: shipped TunableOp results)")
    args = ap.parse_args()

    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.llama import Llama, LlamaConfig
    from llm_training_amd.ops.native import lib
    from llm_training_amd.parallel.context import ParallelContext, init_distributed
    from llm_training_amd.parallel.engine import DataParallelEngine
    from llm_training_amd.runtime.gemm_tuning import setup_gemm_tuning

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
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    lib()  # fail loudly if the HIP extension is missing
    pc = ParallelContext.create("auto", args.tp, device)
    cfg = dict(LLAMA3_8B)
    if args.layers:
        cfg["num_hidden_layers"] = args.layers
    mcfg = LlamaConfig(**cfg, attn_implementation=args.attn, enable_gradient_checkpointing=args.ckpt,
                       loss_chunk_size=args.loss_chunk)
    torch.manual_seed(1234)
    model = Llama(mcfg, pc, dtype=torch.bfloat16, device=device)
    model.init_weights(seed=1234)
    stage = args.zero_stage if args.zero_stage is not None else (0 if pc.dp_size == 1 else 2)
    engine = DataParallelEngine(model, pc, stage, lr=3e-5, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1,
                                offload_optimizer=args.offload_optimizer, force_sharded=args.force_sharded)
    lm = CLM({"model": None})
    lm.model = model
    lm.train()

    B, S = args.micro_batch, args.seq
    g = torch.Generator(device=device).manual_seed(1000 + pc.dp_rank)

    def make_batch():
        ids = torch.randint(0, cfg["vocab_size"], (B, S), device=device, generator=g)
        return {"input_ids": ids, "labels": ids, "position_ids": torch.arange(S, device=device).expand(B, S),
                "attention_mask": None}

    def step(batch):
        engine.begin_step(1)
        engine.zero_grad()
        engine.begin_micro(0)
        loss, _, _ = lm.training_step(batch)
        loss.backward()
        engine.finish_backward()
        engine.clip_and_scale(1.0)
        engine.step(3e-5)
        return loss

    # fresh synthetic batches for every step (pre-generated so the timed loop does no data work)
    batches = [make_batch() for _ in range(args.warmup + args.steps)]
    for i in range(args.warmup):
        loss = step(batches[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(batches[args.warmup + i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.item()
    final_loss = float(loss.detach().float().item())
    tokens = pc.dp_size * B * S * args.steps
    tps = tokens / el
    fpt = flops_per_token(cfg, S)
    peak_mem = torch.cuda.max_memory_allocated(device) / 2 ** 30
    if rank == 0:
        par = f"dp{pc.dp_size}" + (f"-tp{pc.tp_size}" if pc.tp_size > 1 else "")
        out = {
            "metric": "tokens/sec (whole node) Llama-3-8B CLM pre-train",
            "value": round(tps, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1000, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": "Llama-3-8B" if not args.layers else f"Llama-3-8B-{args.layers}L(INVALID-debug)",
                       "global_batch": pc.dp_size * B, "seq_len": S, "parallelism": par, "zero_stage": stage,
                       "attn": args.attn, "activation_checkpointing": args.ckpt, "optimizer": ("host AdamW (offload) fp32 master" if args.offload_optimizer else "fused AdamW fp32 master"),
                       "grad_clip": 1.0, "gemm_tuning": gemm_mode,
                       **({"force_sharded": True} if args.force_sharded else {})},
            "tokens_per_sec_per_gpu": round(tps / world, 2),
            "mfu": round(tps / world * fpt / 2.5e15, 4),
            "tflops_per_gpu": round(tps / world * fpt / 1e12, 1),
            "peak_mem_gib": round(peak_mem, 1),
            "final_loss": round(final_loss, 4),
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
