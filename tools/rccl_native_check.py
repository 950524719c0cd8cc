"""Multi-GPU check of the native RCCL communicators against torch.distributed (RCCL) on the
same data: world + per-axis split communicators, every collective the engine's data path uses.

    python -m butterfly_amd launch -n 8 -- python tools/rccl_native_check.py dp4xtp2

Needs one GPU per rank (RCCL refuses two ranks on one device). Prints one PASS/FAIL line per
rank and exits non-zero on any mismatch."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from butterfly_amd.parallel.comm import Communicator, init_distributed  # noqa: E402
from butterfly_amd.parallel.mesh import Mesh  # noqa: E402


def parse(spec: str, world: int) -> Mesh:
    axes = {"dp": 1, "pp": 1, "tp": 1}
    for part in spec.split("x"):
        for k in axes:
            if part.startswith(k):
                axes[k] = int(part[len(k):])
    m = Mesh(**axes)
    assert m.world_size == world, (spec, world)
    return m


def main() -> int:
    rank, world, local = init_distributed("nccl")
    torch.cuda.set_device(local)
    mesh = parse(sys.argv[1] if len(sys.argv) > 1 else f"tp{world}", world)
    os.environ["BFLY_NATIVE_RCCL"] = "0"
    comm = Communicator.from_mesh(mesh)
    natives = comm.enable_native_rccl()
    ok = True
    g = torch.Generator().manual_seed(100 + rank)
    for axis, nc in natives.items():
        grp = comm.groups[axis]
        x = torch.randn(64, 8192, generator=g).to(torch.bfloat16).cuda()
        a, b = x.clone(), x.clone()
        nc.all_reduce_(a)
        dist.all_reduce(b, group=grp.pg)
        ok &= torch.equal(a, b)
        out_n = torch.empty(grp.size * 64, 8192, dtype=torch.bfloat16, device="cuda")
        out_t = torch.empty_like(out_n)
        nc.all_gather(x, out_n)
        dist.all_gather_into_tensor(out_t, x, group=grp.pg)
        ok &= torch.equal(out_n, out_t)
        y = torch.randn(grp.size * 32, 1024, generator=g).cuda()
        rs_n = torch.empty(32, 1024, device="cuda")
        rs_t = torch.empty_like(rs_n)
        nc.reduce_scatter(y, rs_n)
        dist.reduce_scatter_tensor(rs_t, y, group=grp.pg)
        ok &= torch.allclose(rs_n, rs_t, rtol=1e-5, atol=1e-5)
        a2_n, a2_t = torch.empty_like(y), torch.empty_like(y)
        nc.all_to_all(y, a2_n)
        dist.all_to_all_single(a2_t, y, group=grp.pg)
        ok &= torch.equal(a2_n, a2_t)
        ok &= nc.async_error() == 0
        print(f"rank {rank} axis {axis} size {grp.size}: {'PASS' if ok else 'FAIL'}", flush=True)
    torch.cuda.synchronize()
    dist.barrier()
    print(f"rank {rank} native rccl {sorted(natives)}: {'PASS' if ok else 'FAIL'}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
