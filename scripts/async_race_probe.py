"""Probe: async-optimizer-stream vs synchronous training difference (tiny Llama, 1 GPU)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_model_gpu import _cfg, _train_engine  # noqa: E402

dev = torch.device("cuda", 0)
for layers in (2, 4):
    cfg = _cfg(num_hidden_layers=layers)
    _, la, pa = _train_engine(cfg, dev, overlap_step=False)
    _, lb, pb = _train_engine(cfg, dev, overlap_step=False)
    _, lc, pc = _train_engine(cfg, dev, overlap_step=True)
    for k in pa:
        dn = (pb[k] - pa[k]).norm().item() / (pa[k].norm().item() + 1e-30)
        da = (pc[k] - pa[k]).norm().item() / (pa[k].norm().item() + 1e-30)
        if da > 1e-5 or dn > 1e-5:
            print(f"L{layers} {k:50s} sync-vs-sync {dn:.2e} async-vs-sync {da:.2e}", flush=True)
    print(f"L{layers} losses", la, lc, flush=True)
