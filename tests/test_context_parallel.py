"""Context-parallel prefill (ring attention + LSE merge, parallel/context_parallel.py) on
CPU/gloo: cp = 2 and 3 ranks with replicated weights must reproduce the single-process prefill
logits, and each rank's paged KV cache must hold exactly its chunk's K/V."""
import pytest
import torch

from butterfly_amd.config import ModelConfig
from butterfly_amd.engine.batch import make_prefill_batch
from butterfly_amd.models import build_model
from butterfly_amd.ops import reference as ref
from butterfly_amd.parallel.context_parallel import split_lengths

from .dist_utils import run_world

PROMPTS = [[(7 * i + 3) % 1000 + 1 for i in range(45)], [5, 9, 2, 77, 31, 8, 8, 100], [42, 43]]
BS = 32


def _model(preset="llama-tiny"):
    cfg = ModelConfig.from_preset(preset)
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    m.init_random(11)
    return m


def _single():
    m = _model()
    kv = m.allocate_kv_cache(8, BS)
    slots, nxt = [], 0
    for p in PROMPTS:
        slots.append(list(range(nxt, nxt + len(p))))
        nxt += ((len(p) + BS - 1) // BS) * BS
    logits = m.forward(make_prefill_batch(PROMPTS, slots), kv)
    return logits, kv, slots


def _cp_rank(rank, world, attn="ring"):
    import torch.distributed as dist

    from butterfly_amd.parallel.context_parallel import cp_prefill

    m = _model()
    kv = m.allocate_kv_cache(8, BS)
    # this rank's chunk of prompt i goes to slots [i*64 + offset of the chunk ...)
    slots = []
    for i, p in enumerate(PROMPTS):
        lens = split_lengths(len(p), world)
        a = sum(lens[:rank])
        slots.append([i * 64 + a + j for j in range(lens[rank])])
    logits = cp_prefill(m, PROMPTS, list(range(world)), rank, dist.group.WORLD, kv, slots, attn=attn)
    # numpy: pickled by value through the result queue (tensors would go by shared memory)
    return logits.numpy(), [(k.numpy(), v.numpy()) for k, v in kv], slots


@pytest.mark.parametrize("world,attn", [(2, "ring"), (3, "ring"), (2, "ulysses")])
def test_cp_prefill_matches_single(world, attn):
    want, kv_ref, slots_ref = _single()
    outs = run_world(_cp_rank, world, attn)
    for logits, kv, slots in outs:
        logits = torch.from_numpy(logits)
        kv = [(torch.from_numpy(k), torch.from_numpy(v)) for k, v in kv]
        assert torch.allclose(logits, want, atol=1e-4, rtol=1e-4), (logits - want).abs().max()
        # the rank's cache holds its chunk's K/V at its slots, equal to the single-run entries
        for (k, v), (kr, vr) in zip(kv, kv_ref):
            for i, sl in enumerate(slots):
                lens = split_lengths(len(PROMPTS[i]), world)
                a = sl[0] - i * 64 if sl else 0
                for j, s in enumerate(sl):
                    t = slots_ref[i][a + j]
                    assert torch.allclose(k[s // BS, :, s % BS], kr[t // BS, :, t % BS], atol=1e-5)
                    assert torch.allclose(v[s // BS, :, :, s % BS], vr[t // BS, :, :, t % BS], atol=1e-5)


def test_lse_merge_of_chunks_equals_full_attention():
    torch.manual_seed(0)
    T, H, Hk, D = 50, 4, 2, 128
    q, k, v = torch.randn(T, H, D), torch.randn(T, Hk, D), torch.randn(T, Hk, D)
    cu = torch.tensor([0, 50], dtype=torch.int32)
    full, lf = ref.attn_prefill(q, k, v, cu, 50, 0.09, True, return_lse=True)
    # queries of rows [30, 50) against keys [0, 30) (visible) then [30, 50) (causal)
    cq = torch.tensor([0, 20], dtype=torch.int32)
    o1, l1 = ref.attn_prefill(q[30:], k[:30], v[:30], cq, 20, 0.09, False,
                              cu_seqlens_k=torch.tensor([0, 30], dtype=torch.int32), return_lse=True)
    o2, l2 = ref.attn_prefill(q[30:], k[30:], v[30:], cq, 20, 0.09, True, return_lse=True)
    acc, al = o2.float().clone(), l2.clone()
    ref.attn_lse_merge_(acc, al, o1, l1)
    assert torch.allclose(acc, full[30:], atol=1e-5) and torch.allclose(al, lf[30:], atol=1e-5)
