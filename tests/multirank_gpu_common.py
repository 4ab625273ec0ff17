"""Shared config of tests/test_multirank_gpu.py and its rank processes."""
import torch

from llm_training_amd.models.llama import LlamaConfig

CFG = LlamaConfig(vocab_size=4096, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                  num_attention_heads=8, num_key_value_heads=4, max_position_embeddings=2048,
                  rope_theta=500000.0)
STEPS = 3


def batches(dev):
    g = torch.Generator().manual_seed(11)
    return [torch.randint(0, CFG.vocab_size, (2, 512), generator=g).to(dev) for _ in range(STEPS)]


def pref_batches(dev, B=2, S=256):
    g = torch.Generator().manual_seed(21)
    out = []
    for _ in range(STEPS):
        b = {}
        for side in ("chosen", "rejected"):
            ids = torch.randint(1, CFG.vocab_size, (B, S), generator=g)
            lab = ids.clone()
            lab[:, :S // 4] = -100
            b.update({f"{side}_input_ids": ids.to(dev), f"{side}_labels": lab.to(dev),
                      f"{side}_attention_mask": torch.ones(B, S, dtype=torch.long, device=dev)})
        out.append(b)
    return out
