#!/usr/bin/env python3
"""Instruction mix of a kernel's hot loop, from the gfx950 assembly hipcc emits (no GPU needed).

Compiles one kernel source with --save-temps, finds the named kernel's body in the device .s
and prints, per basic block holding at least `--min-mfma` MFMAs (the unrolled K / tile loop),
the counts of MFMA, other VALU, SALU, LDS reads / writes, LDS-DMA / buffer loads, waits and
barriers — the numbers to set against PMC counters (SQ_INSTS_VALU counts MFMAs too) when
asking whether a loop is VALU-, LDS- or issue-bound.

usage: python tools/isa_stats.py csrc/kernels/gemm.hip gemm_big8_kernelILb1 [--min-mfma 16] [--md out.md]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def device_asm(src: str, workdir: str) -> str:
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/csrc/include",
           "-c", os.path.abspath(src), "-o", os.path.join(workdir, "k.o"), "--save-temps"]
    subprocess.run(cmd, cwd=workdir, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    s = [f for f in os.listdir(workdir) if f.endswith("gfx950.s")]
    if not s:
        raise SystemExit("no device assembly produced")
    with open(os.path.join(workdir, s[0])) as f:
        return f.read()


def kernel_body(asm: str, pattern: str) -> tuple:
    names = [n for n in re.findall(r"^(_Z\S+):", asm, re.M) if pattern in n]
    if not names:
        raise SystemExit(f"no kernel symbol contains {pattern!r}")
    name = names[0]
    i = asm.index(name + ":")
    j = asm.index(".Lfunc_end", i)
    return name, asm[i:j].split("\n")


CLASSES = (
    ("mfma", lambda op: op.startswith("v_mfma")),
    ("valu", lambda op: op.startswith("v_") and not op.startswith("v_mfma")),
    ("salu", lambda op: op.startswith("s_") and not op.startswith(("s_waitcnt", "s_barrier", "s_load", "s_buffer"))),
    ("smem", lambda op: op.startswith(("s_load", "s_buffer_load"))),
    ("ds_read", lambda op: op.startswith("ds_read")),
    ("ds_write", lambda op: op.startswith("ds_write")),
    ("vmem_lds", lambda op: op.startswith(("global_load_lds", "buffer_load")) and "lds" in op),
    ("vmem_load", lambda op: op.startswith(("global_load", "buffer_load")) and "lds" not in op),
    ("vmem_store", lambda op: op.startswith(("global_store", "buffer_store"))),
    ("waitcnt", lambda op: op.startswith("s_waitcnt")),
    ("barrier", lambda op: op.startswith("s_barrier")),
)


def block_stats(lines):
    c = collections.Counter()
    valu_ops = collections.Counter()
    for ln in lines:
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        for cls, pred in CLASSES:
            if pred(op):
                c[cls] += 1
                if cls == "valu":
                    valu_ops[op] += 1
                break
    return c, valu_ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--min-mfma", type=int, default=16)
    ap.add_argument("--md", default=None)
    ap.add_argument("--span", action="store_true",
                    help="also count the blocks between the first and last hot block (the loop's MFMA-free phases)")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as wd:
        asm = device_asm(a.src, wd)
    name, body = kernel_body(asm, a.kernel)
    starts = [k for k, ln in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", ln)] + [len(body)]
    rows, total = [], collections.Counter()
    top = collections.Counter()
    blocks = list(zip(starts, starts[1:]))
    hot = [i for i, (s, e) in enumerate(blocks) if block_stats(body[s:e])[0]["mfma"] >= a.min_mfma]
    for i, (s, e) in enumerate(blocks):
        c, ops = block_stats(body[s:e])
        if c["mfma"] >= a.min_mfma or (a.span and hot and hot[0] <= i <= hot[-1]):
            rows.append((body[s].split(":")[0], c))
            total.update(c)
            top.update(ops)
    cols = [k for k, _ in CLASSES]
    out = [f"# {name}", "", f"basic blocks with >= {a.min_mfma} MFMAs (the hot loop, unrolled)" + (" and every block between them" if a.span else ""), "",
           "| block | " + " | ".join(cols) + " |", "|---" * (len(cols) + 1) + "|"]
    for lab, c in rows:
        out.append(f"| {lab} | " + " | ".join(str(c[k]) for k in cols) + " |")
    out.append("| **sum** | " + " | ".join(str(total[k]) for k in cols) + " |")
    out += ["", "most frequent VALU ops in those blocks: " + ", ".join(f"{o} x{n}" for o, n in top.most_common(10))]
    text = "\n".join(out) + "\n"
    if a.md:
        with open(a.md, "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
