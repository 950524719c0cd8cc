"""ForwardBatch: the device-side description of one model step (prefill or decode)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class ForwardBatch:
    input_ids: torch.Tensor                 # int32 [T]
    positions: torch.Tensor                 # int32 [T]
    slots: torch.Tensor                     # int32 [T] paged-cache slot per token (-1 = none)
    is_prefill: bool
    # prefill: sequences packed back to back
    cu_seqlens: Optional[torch.Tensor] = None   # int32 [nseq + 1]
    max_seqlen: int = 0
    # decode: one token per sequence
    block_tables: Optional[torch.Tensor] = None  # int32 [B, max_blocks]
    ctx_lens: Optional[torch.Tensor] = None      # int32 [B] context length incl. the new token
    max_ctx: int = 0                             # static upper bound of ctx_lens
    logits_idx: Optional[torch.Tensor] = None    # int64 [R] rows that need logits (None = all)
    ep_tokens: int = 0                           # EP: token rows every rank pads to (0 = no pad)
    ep_alltoall: bool = False                    # EP: this step dispatches tokens by all-to-all
    cp: Optional[object] = None                  # prefill over a context-parallel group (CPContext)
    # mixed steps (chunked prefill + decode): the first num_decode rows are decode rows
    # (block_tables / ctx_lens / max_ctx describe them); the remaining rows are prompt chunks
    # (cu_seqlens over them). A chunk starting at position p > 0 also attends to the p tokens
    # already cached: prefix_lens (host list), prefix_cu (device cumsum), prefix_tables.
    num_decode: int = 0
    prefix_lens: Optional[list] = None
    prefix_cu: Optional[torch.Tensor] = None
    prefix_tables: Optional[torch.Tensor] = None
    # when the chunks with a cached prefix are the leading `split_seqs` chunks (split_rows rows)
    # and the rest are fresh prompts: the fresh ones take the flash kernel (cu_fresh over them)
    split_seqs: int = 0
    split_rows: int = 0
    cu_fresh: Optional[torch.Tensor] = None
    max_fresh: int = 0
    max_paged: int = 0

    @property
    def num_tokens(self) -> int:
        return int(self.input_ids.shape[0])

    @property
    def num_seqs(self) -> int:
        if self.is_prefill:
            return int(self.cu_seqlens.shape[0]) - 1
        return int(self.ctx_lens.shape[0])

    def to(self, device) -> "ForwardBatch":
        mv = lambda t: None if t is None else t.to(device, non_blocking=True)  # noqa: E731
        return ForwardBatch(mv(self.input_ids), mv(self.positions), mv(self.slots), self.is_prefill,
                            mv(self.cu_seqlens), self.max_seqlen, mv(self.block_tables),
                            mv(self.ctx_lens), self.max_ctx, mv(self.logits_idx), self.ep_tokens,
                            self.ep_alltoall, self.cp, self.num_decode, self.prefix_lens,
                            mv(self.prefix_cu), mv(self.prefix_tables), self.split_seqs, self.split_rows,
                            mv(self.cu_fresh), self.max_fresh, self.max_paged)


def make_prefill_batch(prompts: list[list[int]], slots: list[list[int]], device="cpu",
                       start_positions: Optional[list[int]] = None) -> ForwardBatch:
    """Pack prompts back to back. `slots[i][j]` = cache slot of token j of prompt i."""
    ids, pos, sl, cu = [], [], [], [0]
    for i, p in enumerate(prompts):
        s0 = start_positions[i] if start_positions else 0
        ids.extend(p)
        pos.extend(range(s0, s0 + len(p)))
        sl.extend(slots[i])
        cu.append(cu[-1] + len(p))
    last = [c - 1 for c in cu[1:]]
    i32 = dict(dtype=torch.int32, device=device)
    return ForwardBatch(
        input_ids=torch.tensor(ids, **i32), positions=torch.tensor(pos, **i32),
        slots=torch.tensor(sl, **i32), is_prefill=True, cu_seqlens=torch.tensor(cu, **i32),
        max_seqlen=max(len(p) for p in prompts),
        logits_idx=torch.tensor(last, dtype=torch.int64, device=device))


def make_decode_batch(tokens: list[int], positions: list[int], slots: list[int],
                      block_tables: list[list[int]], max_blocks: int, max_ctx: int,
                      device="cpu") -> ForwardBatch:
    B = len(tokens)
    bt = torch.zeros(B, max_blocks, dtype=torch.int32)
    for i, row in enumerate(block_tables):
        bt[i, : len(row)] = torch.tensor(row, dtype=torch.int32)
    i32 = dict(dtype=torch.int32, device=device)
    return ForwardBatch(
        input_ids=torch.tensor(tokens, **i32), positions=torch.tensor(positions, **i32),
        slots=torch.tensor(slots, **i32), is_prefill=False, block_tables=bt.to(device),
        ctx_lens=torch.tensor([p + 1 for p in positions], **i32), max_ctx=max_ctx,
        logits_idx=None)


def empty_batch(device="cpu", ep_tokens: int = 0) -> ForwardBatch:
    """A zero-token step: lets an idle expert-parallel rank join its peers' collectives."""
    i32 = dict(dtype=torch.int32, device=device)
    return ForwardBatch(input_ids=torch.zeros(0, **i32), positions=torch.zeros(0, **i32),
                        slots=torch.zeros(0, **i32), is_prefill=True,
                        cu_seqlens=torch.zeros(1, **i32), max_seqlen=0,
                        logits_idx=torch.zeros(0, dtype=torch.int64, device=device), ep_tokens=ep_tokens)
