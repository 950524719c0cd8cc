#!/usr/bin/env python3
"""Diagnosis of the round-3 Llama-3-70B tp4 shared-GPU rehearsal stall.

Hypothesis: co-residency starvation. N ranks share ONE GPU; the IPC all-reduce's 128
workgroups of an early rank spin on flags while a late rank's preceding GEMM still needs whole
CUs (one 512-thread workgroup with most of a CU's VGPRs / LDS): the spinners hold resources
the GEMM workgroups wait for, so the late rank's all-reduce starts only when the spinners give
up (20 s flag-wait limit), with the sticky error word set. On separate GPUs nothing competes
for a rank's CUs, so the same protocol cannot starve.

Experiment (every rank on cuda:0, gloo only for the setup): rank 0 issues the all-reduce at
once; ranks 1..N-1 first queue `--gemms` large prefill GEMMs (the 70B gate/up shape), then the
same all-reduce. Reported per rank: wall time of its queue, the device error word and the
host-mapped health word. Control: every rank queues the GEMMs first (no early spinner).
A starved run shows ~20 s and error words set; a healthy protocol finishes in the GEMM time.

Variant --late 1: three early spinners, one late rank (the round-3 rehearsal's pattern): the
spinners hold every CU, the late rank's GEMM cannot be placed until they give up.

usage: python -m butterfly_amd launch -n 4 -- python tools/car_starve.py [--two-shot] [--control] [--late N]
"""
import argparse
import os
import sys
import time

os.environ.setdefault("BFLY_IPC_SHARED_DEVICE", "1")     # the point of the experiment
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--two-shot", action="store_true")
    ap.add_argument("--control", action="store_true", help="every rank queues the GEMMs first")
    ap.add_argument("--gemms", type=int, default=12)
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--late", type=int, default=None,
                    help="ranks that queue the GEMMs before the all-reduce (the LAST ones; default all but rank 0)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from butterfly_amd import ops
    from butterfly_amd.parallel.custom_allreduce import CustomAllReduce

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    car = CustomAllReduce(list(range(world)), rank, dist.group.WORLD, max_bytes=8 << 20, device=dev)
    if not car.ok:
        print(f"rank {rank}: custom all-reduce self-test failed", flush=True)
        return 2
    x = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
    w = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
    ops.linear(x, w)                                  # warm the GEMM path
    t = torch.full((a.rows, 8192), float(rank + 1), dtype=torch.bfloat16, device=dev)
    torch.cuda.synchronize()
    t_gemm = time.perf_counter()
    for _ in range(a.gemms):
        ops.linear(x, w)
    torch.cuda.synchronize()
    gemm_s = time.perf_counter() - t_gemm
    car.clear_error()
    torch.ops.bfly.health_clear()
    dist.barrier()
    t0 = time.perf_counter()
    late = world - 1 if a.late is None else a.late
    if rank >= world - late or a.control:
        for _ in range(a.gemms):
            ops.linear(x, w)
    car.all_reduce_(t, two_shot=a.two_shot)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = bool((t.float() == sum(range(1, world + 1))).all())
    print(f"STARVE rank={rank} world={world} late={late} two_shot={a.two_shot} control={a.control} rows={a.rows} "
          f"gemm_queue_alone={gemm_s * 1e3:.1f}ms wall={dt * 1e3:.1f}ms err_word={car.error()} "
          f"health_words={list(torch.ops.bfly.health_words())} result_ok={ok}", flush=True)
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
