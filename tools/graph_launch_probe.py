#!/usr/bin/env python3
"""Does hipGraphLaunch return before the graph has run? Host time spent inside `replay()` for a
captured graph of `--kernels` kernels (each a ~20-50 us elementwise pass over `--mb` MiB), next
to the graph's GPU time. A launch that returns in far less than the GPU time leaves the host
free to prepare the next step while the device works (the asynchronous engine relies on that).

usage: python tools/graph_launch_probe.py [--kernels 400,650] [--mb 64] [--replays 6]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="100,400,650,1000")
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--replays", type=int, default=6)
    a = ap.parse_args()
    x = torch.zeros(a.mb << 18, device="cuda")          # mb MiB of f32
    for n in map(int, a.kernels.split(",")):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(n):
                x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                x.add_(1.0)
        g.replay()
        torch.cuda.synchronize()
        host, gpu = [], []
        for _ in range(a.replays):
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            t = time.perf_counter()
            g.replay()
            host.append((time.perf_counter() - t) * 1e3)
            en.record()
            torch.cuda.synchronize()
            gpu.append(st.elapsed_time(en))
        # back to back: the second launch while the first still runs
        t = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        g.replay()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        print(json.dumps({"kernels": n, "gpu_ms": round(sorted(gpu)[len(gpu) // 2], 3),
                          "host_ms_in_replay": round(sorted(host)[len(host) // 2], 3),
                          "back_to_back_host_ms": [round((t1 - t) * 1e3, 3), round((t2 - t1) * 1e3, 3)]}),
              flush=True)
        del g


if __name__ == "__main__":
    main()
