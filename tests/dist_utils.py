"""Multi-process CPU harness: spawn `world` ranks on gloo (127.0.0.1) and collect results."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import torch
        import torch.distributed as dist

        torch.set_num_threads(max(1, 8 // world))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))


def run_world(fn, world: int, *args, timeout: float = 300.0):
    """Run fn(rank, world, *args) on `world` gloo ranks; returns results ordered by rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{res}")
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]
