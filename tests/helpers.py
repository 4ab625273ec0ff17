"""Shared test utilities (toy tokenizer, tiny configs, gloo multi-process launcher)."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp


def toy_tokenizer(extra_words=()):
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast

    words = ("hello world how are you user assistant system fine thanks the a of to and is it in that "
             "good bad yes no maybe question answer").split() + list(extra_words)
    tk = Tokenizer(models.WordLevel(unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    tr = trainers.WordLevelTrainer(special_tokens=["<unk>", "<pad>", "<s>", "</s>", "<|im_start|>", "<|im_end|>",
                                                   "<|user|>", "<|assistant|>", "<|end|>", "<|system|>"])
    tk.train_from_iterator([" ".join(words)], tr)
    return PreTrainedTokenizerFast(tokenizer_object=tk, bos_token="<s>", eos_token="</s>", pad_token="<pad>",
                                   unk_token="<unk>")


def tiny_llama_cfg(**kw):
    from llm_training_amd.models.llama import LlamaConfig

    d = dict(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
             num_key_value_heads=2, max_position_embeddings=256)
    d.update(kw)
    return LlamaConfig(**d)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import io
        res = fn(rank, world, *args)
        buf = io.BytesIO()
        torch.save(res, buf)  # plain bytes: no shared-memory handles outliving this process
        q.put((rank, "ok", buf.getvalue()))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def run_gloo(fn, world=2, args=(), timeout=240):
    """Run fn(rank, world, *args) in `world` gloo processes; return {rank: result}."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            import io
            out[rank] = torch.load(io.BytesIO(res), weights_only=True)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out
