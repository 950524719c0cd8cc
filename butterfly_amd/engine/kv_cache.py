"""Paged KV cache of one rank: device tensors + the C++ page manager.

Layout per local layer (models/transformer.py allocate_kv_cache):
  K [num_blocks, kv_heads_local, block_size, head_dim]   (rows contiguous: QK^T operand)
  V [num_blocks, kv_heads_local, head_dim, block_size]   (transposed: PV operand)
Elements are the model dtype or, with EngineConfig.kv_cache_dtype="fp8", FP8 e4m3
(torch.float8_e4m3fn, written and read by the HIP kernels: csrc/include/bfly_kv.h).
Capacity is sized from the HBM left after weights and activations (SURVEY.md §2.7 A14:
"KV-cache shards sized for 288 GB HBM3E"): on one MI355X a Llama-3-70B shard leaves ~130 GB
for KV, ~400 k tokens; with TP=8 each rank keeps 1/8 of the kv heads, so capacity per token
grows 8x.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native_loader


def kv_blocks_for_budget(bytes_budget: int, bytes_per_token: int, block_size: int) -> int:
    per_block = bytes_per_token * block_size
    return max(0, bytes_budget // per_block)


def device_kv_budget(device: torch.device, utilization: float, reserve_bytes: int = 0) -> int:
    """Bytes available for KV on `device` after what is already allocated (weights etc.)."""
    if device.type != "cuda":
        return 1 << 30
    free, total = torch.cuda.mem_get_info(device)
    allowed = int(total * utilization) - (total - free) - reserve_bytes
    return max(0, allowed)


class KVCache:
    def __init__(self, model, num_blocks: int, block_size: int, dtype: Optional[torch.dtype] = None):
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.layers = model.allocate_kv_cache(num_blocks, block_size, dtype)
        self.dtype = self.layers[0][0].dtype if self.layers else dtype
        native = _native_loader.native()
        self.manager = native.KVBlockManager(num_blocks, block_size)

    @property
    def capacity_tokens(self) -> int:
        return self.num_blocks * self.block_size

    def bytes(self) -> int:
        return sum(k.numel() * k.element_size() + v.numel() * v.element_size() for k, v in self.layers)

    def copy_blocks(self, pairs: list) -> None:
        """Copy-on-write page copies (src -> dst) before a step that writes to a forked page."""
        for src, dst in pairs:
            for k, v in self.layers:
                k[dst].copy_(k[src])
                v[dst].copy_(v[src])
