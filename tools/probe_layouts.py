import torch, sys
sys.path.insert(0, '.')
from butterfly_amd import ops
ops.load_library()
out = torch.zeros(64*16, device='cuda')
for w in (3, 4):
    out.zero_(); torch.ops.bfly.probe(w, out); torch.cuda.synchronize()
    o = out[:512].view(64, 8).cpu().long()
    print("probe", w, "(3: rows, 4: cols)")
    for l in range(64):
        print(l, o[l].tolist())
