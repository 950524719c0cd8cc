"""HuggingFace checkpoint import: Llama / Mistral / Mixtral / GPT-2 safetensors -> butterfly-ckpt.

Maps HF parameter names to our logical names (the names `TransformerLM.logical_params()`
uses) and converts layouts (GPT-2's Conv1D weights are stored [in, out] and its attention is
one fused c_attn; both are split/transposed here). The output is a single-writer checkpoint
whose tensors are whole (split_dim = null), which any PartitionPlan can load (resharding
happens at load time, ckpt/format.py).
"""
from __future__ import annotations

import json
import re
from pathlib import Path
from typing import Iterator

import torch
from safetensors import safe_open
from safetensors.torch import save_file

from ..config import ModelConfig
from .format import _DT, FORMAT, VERSION

_LLAMA = [
    (r"model\.embed_tokens\.weight", "embed_tokens.weight"),
    (r"model\.norm\.weight", "final_norm.weight"),
    (r"lm_head\.weight", "lm_head.weight"),
    (r"model\.layers\.(\d+)\.input_layernorm\.weight", r"layers.\1.input_norm.weight"),
    (r"model\.layers\.(\d+)\.post_attention_layernorm\.weight", r"layers.\1.post_norm.weight"),
    (r"model\.layers\.(\d+)\.self_attn\.(q|k|v|o)_proj\.weight", r"layers.\1.attn.\2_proj.weight"),
    (r"model\.layers\.(\d+)\.mlp\.(gate|up|down)_proj\.weight", r"layers.\1.mlp.\2_proj.weight"),
    (r"model\.layers\.(\d+)\.block_sparse_moe\.gate\.weight", r"layers.\1.moe.router.weight"),
    (r"model\.layers\.(\d+)\.block_sparse_moe\.experts\.(\d+)\.w1\.weight", r"layers.\1.moe.experts.\2.gate_proj.weight"),
    (r"model\.layers\.(\d+)\.block_sparse_moe\.experts\.(\d+)\.w3\.weight", r"layers.\1.moe.experts.\2.up_proj.weight"),
    (r"model\.layers\.(\d+)\.block_sparse_moe\.experts\.(\d+)\.w2\.weight", r"layers.\1.moe.experts.\2.down_proj.weight"),
]


def _llama_map(name: str, t: torch.Tensor) -> Iterator[tuple[str, torch.Tensor]]:
    for pat, rep in _LLAMA:
        if re.fullmatch(pat, name):
            yield re.sub(pat, rep, name), t
            return


def _gpt2_map(name: str, t: torch.Tensor, h: int) -> Iterator[tuple[str, torch.Tensor]]:
    n = name[len("transformer."):] if name.startswith("transformer.") else name
    if n == "wte.weight":
        yield "embed_tokens.weight", t
    elif n == "wpe.weight":
        yield "pos_embed.weight", t
    elif n in ("ln_f.weight", "ln_f.bias"):
        yield "final_norm." + n.split(".")[1], t
    else:
        m = re.fullmatch(r"h\.(\d+)\.(.+)", n)
        if not m:
            return
        i, rest = m.group(1), m.group(2)
        L = f"layers.{i}."
        if rest.startswith("ln_1."):
            yield L + "input_norm." + rest[5:], t
        elif rest.startswith("ln_2."):
            yield L + "post_norm." + rest[5:], t
        elif rest == "attn.c_attn.weight":       # Conv1D [h, 3h]
            q, k, v = t.t().split(h, 0)
            yield L + "attn.q_proj.weight", q
            yield L + "attn.k_proj.weight", k
            yield L + "attn.v_proj.weight", v
        elif rest == "attn.c_attn.bias":
            q, k, v = t.split(h, 0)
            yield L + "attn.q_proj.bias", q
            yield L + "attn.k_proj.bias", k
            yield L + "attn.v_proj.bias", v
        elif rest == "attn.c_proj.weight":
            yield L + "attn.o_proj.weight", t.t()
        elif rest == "attn.c_proj.bias":
            yield L + "attn.o_proj.bias", t
        elif rest == "mlp.c_fc.weight":
            yield L + "mlp.fc.weight", t.t()
        elif rest == "mlp.c_fc.bias":
            yield L + "mlp.fc.bias", t
        elif rest == "mlp.c_proj.weight":
            yield L + "mlp.proj.weight", t.t()
        elif rest == "mlp.c_proj.bias":
            yield L + "mlp.proj.bias", t


def iter_hf_tensors(src: Path) -> Iterator[tuple[str, torch.Tensor]]:
    files = sorted(src.glob("*.safetensors"))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {src}")
    for f in files:
        with safe_open(str(f), framework="pt", device="cpu") as fh:
            for k in fh.keys():
                yield k, fh.get_tensor(k)


def convert_hf(src: str | Path, dst: str | Path, dtype: torch.dtype = torch.bfloat16,
               name: str = "hf") -> ModelConfig:
    """Convert a HuggingFace model directory (config.json + *.safetensors) to butterfly-ckpt.

    Streams one HF shard at a time: each input file becomes one output file
    (`hf-NNNNN.safetensors`), so peak host memory is one shard (~5 GB for the 70B release),
    not the whole model (~141 GB). The manifest points every logical tensor at its file.
    """
    src, dst = Path(src), Path(dst)
    hf_cfg = json.loads((src / "config.json").read_text())
    cfg = ModelConfig.from_hf(hf_cfg, name=name)
    files = sorted(src.glob("*.safetensors"))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {src}")
    dst.mkdir(parents=True, exist_ok=True)
    tensors: dict[str, dict] = {}

    def _write(fname: str, out: dict[str, torch.Tensor]) -> None:
        save_file(out, str(dst / fname), metadata={"format": FORMAT, "source": "huggingface"})
        for n, t in out.items():
            tensors[n] = {"shape": list(t.shape), "dtype": _DT[t.dtype],
                          "shards": [{"file": fname, "split_dim": None, "offset": 0,
                                      "length": t.shape[0]}]}

    for i, f in enumerate(files):
        out: dict[str, torch.Tensor] = {}
        with safe_open(str(f), framework="pt", device="cpu") as fh:
            for k in fh.keys():
                t = fh.get_tensor(k)
                it = _gpt2_map(k, t, cfg.hidden_size) if cfg.arch == "gpt2" else _llama_map(k, t)
                for ln, tt in it:
                    if ln == "lm_head.weight" and cfg.tie_embeddings:
                        continue
                    out[ln] = tt.to(dtype).contiguous()
        if out:
            _write(f"hf-{i:05d}.safetensors", out)
        del out
    if not cfg.tie_embeddings and "lm_head.weight" not in tensors and "embed_tokens.weight" in tensors:
        ef = tensors["embed_tokens.weight"]["shards"][0]["file"]
        with safe_open(str(dst / ef), framework="pt", device="cpu") as fh:
            _write("hf-lm_head.safetensors", {"lm_head.weight": fh.get_tensor("embed_tokens.weight")})
    manifest = {"format": FORMAT, "version": VERSION, "model": cfg.to_dict(), "plan": {},
                "dtype": _DT[dtype], "tensors": tensors}
    (dst / "manifest.json").write_text(json.dumps(manifest, indent=1))
    return cfg
