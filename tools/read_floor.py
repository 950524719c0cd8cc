#!/usr/bin/env python3
"""HBM read floor for single-kernel streams of decode-projection size (16-160 MiB): how long
one launch takes to read N bytes cold, for several grid sizes and loads in flight per lane
(`tools/probes/read_floor.hip`, built with `hipcc --genco --offload-arch=gfx950`). The best
time per size is the floor a decode GEMM of that weight size could reach in one launch.

usage: python tools/read_floor.py [--mib 16,32,48,112,160]
"""
import argparse
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", default="16,32,48,112,160")
    ap.add_argument("--grids", default="256,512,1024,2048,4096")
    ap.add_argument("--tiled", default="6144x4096,4096x4096,4096x14336,10240x8192,8192x8192",
                    help="GEMM-shaped walks over these [N x K] weights ('' = skip)")
    a = ap.parse_args()
    co = os.path.join(HERE, "probes", "read_floor.hsaco")
    if not os.path.exists(co):   # git-ignored build product: compile it (gfx950, no GPU needed)
        subprocess.run(["hipcc", "--genco", "--offload-arch=gfx950", "-O3", co[:-6] + ".hip", "-o", co], check=True)
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    mod, fns = ctypes.c_void_p(), {}
    assert hip.hipModuleLoad(ctypes.byref(mod), co.encode()) == 0
    for name in ("read4", "read8", "read16", "tiled128", "tiled64", "tiled32", "frag1", "frag2", "frag4"):
        f = ctypes.c_void_p()
        assert hip.hipModuleGetFunction(ctypes.byref(f), mod, name.encode()) == 0
        fns[name] = f
    pool = torch.empty(2 << 30, dtype=torch.uint8, device="cuda").fill_(1)
    sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch(f, grid, ptr, n16):
        p, n, k = ctypes.c_void_p(ptr), ctypes.c_long(n16), ctypes.c_void_p(sink.data_ptr())
        args = (ctypes.c_void_p * 3)(ctypes.addressof(p), ctypes.addressof(n), ctypes.addressof(k))
        assert hip.hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, stream, args, None) == 0

    def launch_tiled(f, grid, ptr, n, k, sk):
        p, a1, a2, a3, kk = (ctypes.c_void_p(ptr), ctypes.c_int(n), ctypes.c_int(k), ctypes.c_int(sk),
                             ctypes.c_void_p(sink.data_ptr()))
        args = (ctypes.c_void_p * 5)(*[ctypes.addressof(v) for v in (p, a1, a2, a3, kk)])
        assert hip.hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, stream, args, None) == 0

    def time_it(fn, slots):
        for i in range(4):
            fn(i % slots)
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for i in range(40):
            fn(i % slots)
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / 40 * 1e3

    for shape in filter(None, a.tiled.split(",")):
        N, K = map(int, shape.split("x"))
        nb = N * K * 2
        slots = (2 << 30) // nb
        best = None
        variants = [(f"tiled{bn}", bn) for bn in (128, 64, 32)] + [(f"frag{t}", 16 * t) for t in (1, 2, 4)]
        for kname, bn in variants:
            for sk in (1, 2, 3, 4, 6, 8, 12, 16):
                grid = N // bn * sk
                if grid < 128 or grid > 8192 or (K // 128) // (4 * sk) < 1:
                    continue
                us = time_it(lambda s: launch_tiled(fns[kname], grid, pool.data_ptr() + s * nb, N, K, sk), slots)
                row = {"shape": shape, "MiB": nb >> 20, "kernel": kname, "BN": bn, "splitk": sk, "grid": grid,
                       "us": round(us, 2), "TBps": round(nb / us / 1e6, 2)}
                print(json.dumps(row), flush=True)
                if best is None or us < best["us"]:
                    best = row
        print(json.dumps({"best_tiled": best}), flush=True)

    for mib in map(int, a.mib.split(",")):
        nb = mib << 20
        slots = (2 << 30) // nb
        best = None
        for name, f in fns.items():
            if not name.startswith("read"):
                continue
            for grid in map(int, a.grids.split(",")):
                for i in range(4):
                    launch(f, grid, pool.data_ptr() + (i % slots) * nb, nb // 16)
                torch.cuda.synchronize()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                iters = 40
                st.record()
                for i in range(iters):
                    launch(f, grid, pool.data_ptr() + (i % slots) * nb, nb // 16)
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) / iters * 1e3
                row = {"MiB": mib, "kernel": name, "grid": grid, "us": round(us, 2), "TBps": round(nb / us / 1e6, 2)}
                print(json.dumps(row), flush=True)
                if best is None or us < best["us"]:
                    best = row
        print(json.dumps({"best": best}), flush=True)


if __name__ == "__main__":
    main()
