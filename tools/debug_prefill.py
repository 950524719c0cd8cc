import torch, math, sys
sys.path.insert(0, '.')
from butterfly_amd import ops
from butterfly_amd.ops import reference as ref
torch.manual_seed(0)
dev='cuda'
def run(name, L, causal, q, k, v):
    cu = torch.tensor([0, L], dtype=torch.int32, device=dev)
    o = ops.attn_prefill(q, k, v, cu, L, 0.1, causal)
    r = ref.attn_prefill(q, k, v, cu, L, 0.1, causal)
    err = (o.float() - r.float()).abs()
    print(f"{name}: L={L} causal={causal} maxerr={err.max().item():.4f} mean={err.mean().item():.4f}")
    return o, r
D=128
for L in (32, 64, 65, 128):
    for causal in (False, True):
        q = torch.randn(L,1,D,device=dev).bfloat16(); k = torch.randn(L,1,D,device=dev).bfloat16(); v = torch.randn(L,1,D,device=dev).bfloat16()
        run("rand", L, causal, q, k, v)
L=64
q = torch.zeros(L,1,D,device=dev).bfloat16(); k = torch.randn(L,1,D,device=dev).bfloat16()
v = torch.arange(L,device=dev).float().view(L,1,1).expand(L,1,D).contiguous().bfloat16()
o,r = run("q0_vkey", L, False, q, k, v)
print("o[0,0,:8]", o[0,0,:8].tolist(), "ref", r[0,0,:8].tolist())
v = torch.arange(D,device=dev).float().view(1,1,D).expand(L,1,D).contiguous().bfloat16()
o,r = run("q0_vd", L, False, q, k, v)
print("o[0,0,:16]", o[0,0,:16].tolist())
print("o[5,0,:16]", o[5,0,:16].tolist())
q = torch.randn(L,1,D,device=dev).bfloat16()
v = torch.arange(L,device=dev).float().view(L,1,1).expand(L,1,D).contiguous().bfloat16()
o,r = run("qr_vkey", L, False, q, k, v)
print("o[:8,0,0]", o[:8,0,0].tolist()); print("r[:8,0,0]", r[:8,0,0].tolist())
print("o[3,0,:8]", o[3,0,:8].tolist())
