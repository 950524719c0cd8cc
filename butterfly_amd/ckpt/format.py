"""Sharded checkpoint format ("butterfly-ckpt", version 1) with load-time resharding.

The reference names a checkpoint capability but defines no format, so
this is ours:

  ckpt/
    manifest.json            {"format": "butterfly-ckpt", "version": 1,
                              "model": {...ModelConfig...}, "plan": {...mesh + stages...},
                              "dtype": "bf16",
                              "tensors": {logical_name: {"shape": [...], "dtype": "bf16",
                                          "shards": [{"file": "rank-00003.safetensors",
                                                      "split_dim": 0, "offset": 4096,
                                                      "length": 1024}, ...]}}}
    rank-00000.safetensors   each rank's local slices of the LOGICAL (HF-style) tensors
    ...

Tensors are stored under their logical names with global shapes recorded in the manifest,
never in a fused or padded local layout, so a checkpoint written under one PartitionPlan
loads under any other: `load_into` asks every logical parameter of the target shard for
its global slice and assembles it from whichever saved shards overlap it (partial reads
through safetensors' memory-mapped slices). Replicated tensors are written once (owner rank).
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional

import torch
from safetensors import safe_open
from safetensors.torch import save_file

from ..config import ModelConfig

FORMAT = "butterfly-ckpt"
VERSION = 1
_DT = {torch.bfloat16: "bf16", torch.float16: "f16", torch.float32: "f32"}
_DT_INV = {v: k for k, v in _DT.items()}


def _rank_file(rank: int) -> str:
    return f"rank-{rank:05d}.safetensors"


def _write_rank(model, path: Path, rank: int, dtype: Optional[torch.dtype]) -> None:
    tensors, index = {}, {}
    for lp in model.logical_params():
        if not lp.owner or (lp.split_dim is not None and lp.length == 0):
            continue
        t = lp.get()
        if dtype is not None:
            t = t.to(dtype)
        t = t.detach().contiguous().cpu()
        tensors[lp.name] = t
        index[lp.name] = {"shape": list(lp.global_shape), "dtype": _DT[t.dtype], "split_dim": lp.split_dim,
                          "offset": lp.offset if lp.split_dim is not None else 0,
                          "length": lp.length if lp.split_dim is not None else lp.global_shape[0]}
    save_file(tensors, str(path / _rank_file(rank)), metadata={"format": FORMAT, "rank": str(rank)})
    (path / f"rank-{rank:05d}.index.json").write_text(json.dumps(index))


def _write_manifest(path: Path, world: int, cfg: ModelConfig, plan: Optional[dict], dtype: str) -> None:
    merged: dict = {}
    for r in range(world):
        idx = json.loads((path / f"rank-{r:05d}.index.json").read_text())
        for name, meta in idx.items():
            e = merged.setdefault(name, {"shape": meta["shape"], "dtype": meta["dtype"], "shards": []})
            e["shards"].append({"file": _rank_file(r), "split_dim": meta["split_dim"],
                                "offset": meta["offset"], "length": meta["length"]})
    manifest = {"format": FORMAT, "version": VERSION, "model": cfg.to_dict(), "plan": plan or {},
                "dtype": dtype, "tensors": merged}
    (path / "manifest.json").write_text(json.dumps(manifest, indent=1))
    for r in range(world):
        (path / f"rank-{r:05d}.index.json").unlink(missing_ok=True)


def save(model, path: str | os.PathLike, rank: int = 0, world: int = 1, comm=None,
         plan: Optional[dict] = None, dtype: Optional[torch.dtype] = None) -> None:
    """Write this rank's owned logical slices; rank 0 merges the per-rank indexes into
    manifest.json after a barrier (collective when world > 1)."""
    path = Path(path)
    path.mkdir(parents=True, exist_ok=True)
    _write_rank(model, path, rank, dtype)
    if comm is not None and world > 1:
        comm.barrier()
    if rank == 0:
        _write_manifest(path, world, model.cfg, plan, _DT.get(dtype or model.dtype, "bf16"))
    if comm is not None and world > 1:
        comm.barrier()


def read_manifest(path: str | os.PathLike) -> dict:
    m = json.loads((Path(path) / "manifest.json").read_text())
    if m.get("format") != FORMAT:
        raise ValueError(f"{path} is not a {FORMAT} checkpoint")
    if m.get("version", 0) > VERSION:
        raise ValueError(f"checkpoint version {m['version']} is newer than supported {VERSION}")
    return m


def model_config(path: str | os.PathLike) -> ModelConfig:
    return ModelConfig.from_dict(read_manifest(path)["model"])


class _Reader:
    def __init__(self, root: Path):
        self.root = root
        self.files: dict = {}

    def slice(self, fname: str, key: str):
        f = self.files.get(fname)
        if f is None:
            f = safe_open(str(self.root / fname), framework="pt", device="cpu")
            self.files[fname] = f
        return f.get_slice(key)


def read_global_slice(manifest: dict, reader: _Reader, name: str, split_dim: Optional[int],
                      offset: int, length: int) -> torch.Tensor:
    """Assemble global[name] restricted to [offset, offset+length) along split_dim (whole
    tensor when split_dim is None) from the saved shards, resharding as needed."""
    meta = manifest["tensors"].get(name)
    if meta is None:
        raise KeyError(f"checkpoint has no tensor {name!r}")
    gshape = meta["shape"]
    if split_dim is None:
        split_dim, offset, length = 0, 0, gshape[0]
    out = torch.empty([length if d == split_dim else s for d, s in enumerate(gshape)],
                      dtype=_DT_INV[meta["dtype"]])
    covered = 0
    for sh in meta["shards"]:
        sd = sh["split_dim"]
        if sd is None:  # replicated full tensor
            sl = reader.slice(sh["file"], name)
            idx = [slice(None)] * len(gshape)
            idx[split_dim] = slice(offset, offset + length)
            out.copy_(sl[tuple(idx)])
            return out
        if sd != split_dim:
            raise ValueError(f"{name}: saved split dim {sd} != requested {split_dim}")
        a = max(offset, sh["offset"])
        b = min(offset + length, sh["offset"] + sh["length"])
        if b <= a:
            continue
        sl = reader.slice(sh["file"], name)
        src = [slice(None)] * len(gshape)
        dst = [slice(None)] * len(gshape)
        src[sd] = slice(a - sh["offset"], b - sh["offset"])
        dst[sd] = slice(a - offset, b - offset)
        out[tuple(dst)] = sl[tuple(src)]
        covered += b - a
    if covered != length:
        raise ValueError(f"{name}: shards cover {covered} of {length} requested rows/cols")
    return out


def load_into(model, path: str | os.PathLike, strict: bool = True) -> list:
    """Fill `model` (any shard of any plan) from a checkpoint. Returns missing names."""
    root = Path(path)
    manifest = read_manifest(root)
    saved_cfg = ModelConfig.from_dict(manifest["model"])
    c = model.cfg
    for k in ("hidden_size", "num_layers", "num_heads", "num_kv_heads", "head_dim", "intermediate_size",
              "vocab_size", "num_experts"):
        if getattr(saved_cfg, k) != getattr(c, k):
            raise ValueError(f"checkpoint {k}={getattr(saved_cfg, k)} != model {getattr(c, k)}")
    reader = _Reader(root)
    missing = []
    with torch.no_grad():
        for lp in model.logical_params():
            if lp.split_dim is not None and lp.length == 0:
                continue
            if lp.name not in manifest["tensors"]:
                missing.append(lp.name)
                continue
            t = read_global_slice(manifest, reader, lp.name, lp.split_dim, lp.offset, lp.length)
            lp.set(t.to(device=model.device, dtype=model.dtype))
    if strict and missing:
        raise KeyError(f"checkpoint is missing {len(missing)} tensors, e.g. {missing[:3]}")
    return missing


def reshard(src: str | os.PathLike, dst: str | os.PathLike, plan) -> None:
    """Offline conversion: rewrite checkpoint `src` for PartitionPlan `plan` (one file per
    rank of the new plan), on the CPU; equivalent to loading under `plan` and saving."""
    from ..models import build_model

    man = read_manifest(src)
    cfg = ModelConfig.from_dict(man["model"])
    dtype = _DT_INV[man["dtype"]]
    dst = Path(dst)
    dst.mkdir(parents=True, exist_ok=True)
    for r in range(plan.n_gpus):
        m = build_model(cfg, plan.shard(r), device="cpu", dtype=dtype)
        load_into(m, src)
        _write_rank(m, dst, r, dtype)
        del m
    _write_manifest(dst, plan.n_gpus, cfg, plan.to_dict(), man["dtype"])
