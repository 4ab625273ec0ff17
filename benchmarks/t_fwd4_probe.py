import os, sys, time, torch
sys.path.insert(0, os.getcwd())
from llm_training_amd.ops import fused as F_
from llm_training_amd.ops import reference as ref
var = sys.argv[1]
B, S, Hq, Hkv = (int(x) for x in sys.argv[2:6])
os.environ["LLMT_FA_FWD_VARIANT"] = var
torch.manual_seed(0)
q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
print("launch", var, B, S, Hq, Hkv, flush=True)
with torch.no_grad():
    o = F_.flash_attention(q, k, v, causal=True)
torch.cuda.synchronize()
print("done", flush=True)
orf = ref.attention(q.float(), k.float(), v.float(), True, None, -1)
print("rel err", float((o.float() - orf).norm() / orf.norm()), flush=True)
