"""Plain-PyTorch reference implementations of every butterfly_amd op.

Two roles:
  * the numerics oracle for the HIP kernels (tests compare each kernel against the fp32
    computation here), and
  * the CPU execution path for the gloo plumbing configuration (SURVEY.md §7.3 item 8:
    the GPU path is HIP-only; the CPU path exists for tests and the CPU/gloo config).

Semantics match the kernels exactly, including in-place side effects and cache layouts:
  k_cache [num_blocks, Hkv, BS, D], v_cache [num_blocks, Hkv, D, BS] (V transposed).
"""
from __future__ import annotations

import math
import struct

import torch
import torch.nn.functional as F

SILU_INTERLEAVE = 16  # gate/up row-group size of the fused SwiGLU weight layout


def rms_norm(x, w, eps, out=None, residual=None):
    if residual is not None:
        residual.copy_((x.float() + residual.float()).to(residual.dtype))
        src = residual
    else:
        src = x
    xf = src.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    y = y.to(x.dtype)
    if out is None:
        return y
    out.copy_(y)
    return out


def layer_norm(x, w, b, eps, out=None, residual=None):
    if residual is not None:
        residual.copy_((x.float() + residual.float()).to(residual.dtype))
        src = residual
    else:
        src = x
    y = F.layer_norm(src.float(), (src.shape[-1],), w.float(), b.float(), eps).to(x.dtype)
    if out is None:
        return y
    out.copy_(y)
    return out


def rope_tables(head_dim: int, max_pos: int, theta: float, scaling: dict | None = None,
                device="cpu"):
    """cos/sin tables [max_pos, head_dim/2] (f32) for the rotate-half convention.

    `scaling` supports the Llama-3.1 "llama3" frequency remap
    ({"type": "llama3", "factor", "low_freq_factor", "high_freq_factor",
      "original_max_position_embeddings"}).
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("type") == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        orig = scaling["original_max_position_embeddings"]
        lo_wl, hi_wl = orig / lo, orig / hi
        wl = 2 * math.pi / inv
        smooth = (orig / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def _rotate(x, cos, sin):
    h = x.shape[-1] // 2
    x0, x1 = x[..., :h].float(), x[..., h:].float()
    return torch.cat([x0 * cos - x1 * sin, x1 * cos + x0 * sin], -1)


def sample_pack(scores, ids):
    return torch.stack([scores.float(), ids.to(torch.float32)], 1)


def sample_merge(allp):
    best = allp[:, :, 0].argmax(0)
    return allp.gather(0, best.view(1, -1, 1).expand(1, -1, 2))[0, :, 1].to(torch.int32)


def gather_rows(src, idx, out):
    """out[i] = src[idx[i]] where idx[i] >= 0; other rows of `out` are left as they are."""
    ok = idx >= 0
    if bool(ok.all()):
        out.copy_(src.index_select(0, idx.long()))
    else:
        rows = ok.nonzero().flatten()
        out[rows] = src.index_select(0, idx[rows].long())
    return out


def rope_kv(qkv, positions, cos, sin, n_q, n_kv, slots=None, k_cache=None, v_cache=None):
    T = qkv.shape[0]
    D = qkv.shape[1] // (n_q + 2 * n_kv)
    v3 = qkv.view(T, n_q + 2 * n_kv, D)
    c = cos[positions.long()].unsqueeze(1)
    s = sin[positions.long()].unsqueeze(1)
    rot = _rotate(v3[:, : n_q + n_kv], c, s).to(qkv.dtype)
    v3[:, : n_q + n_kv] = rot
    if slots is not None:
        kv_append(v3[:, n_q: n_q + n_kv], v3[:, n_q + n_kv:], slots, k_cache, v_cache)
    return qkv


def kv_append(k, v, slots, k_cache, v_cache):
    BS = k_cache.shape[2]
    sl = slots.long()
    keep = sl >= 0
    sl = sl[keep]
    blk, off = sl // BS, sl % BS
    k, v = k[keep], v[keep]
    if k_cache.dtype == torch.float8_e4m3fn:   # the kernels clamp to the e4m3 range
        k, v = k.float().clamp(-448, 448), v.float().clamp(-448, 448)
    k_cache[blk, :, off, :] = k.to(k_cache.dtype)
    v_cache[blk, :, :, off] = v.to(v_cache.dtype)


def silu_mul(gu, out=None, interleave=0):
    ffn = gu.shape[-1] // 2
    g, u = split_gate_up(gu, interleave)
    y = (F.silu(g.float()) * u.float()).to(gu.dtype)
    if out is None:
        return y
    out.copy_(y.view(out.shape))
    return out


def split_gate_up(gu, interleave=0):
    ffn = gu.shape[-1] // 2
    if interleave == 0:
        return gu[..., :ffn], gu[..., ffn:]
    lead = gu.shape[:-1]
    r = gu.reshape(*lead, ffn // interleave, 2, interleave)
    return r[..., 0, :].reshape(*lead, ffn), r[..., 1, :].reshape(*lead, ffn)


def interleave_gate_up(gate_w, up_w, group=SILU_INTERLEAVE):
    """[ffn, K] gate and up weights -> [2*ffn, K] rows in alternating `group`-row blocks."""
    ffn, K = gate_w.shape
    g = gate_w.reshape(ffn // group, group, K)
    u = up_w.reshape(ffn // group, group, K)
    return torch.stack([g, u], 1).reshape(2 * ffn, K)


def gelu(x, out=None):
    y = F.gelu(x.float(), approximate="tanh").to(x.dtype)
    if out is None:
        return y
    out.copy_(y)
    return out


def add(a, b, out=None):
    y = (a.float() + b.float()).to(a.dtype)
    if out is None:
        return y
    out.copy_(y)
    return out


def embed(ids, table, vstart=0, out=None):
    local = ids.long() - vstart
    ok = (local >= 0) & (local < table.shape[0])
    y = table[local.clamp(0, table.shape[0] - 1)] * ok.unsqueeze(-1).to(table.dtype)
    if out is None:
        return y
    out.copy_(y.view(out.shape))
    return out


def _mix64(z):
    # splitmix64 finaliser on int64 tensors with wrap-around (matches sample.hip)
    m = (1 << 64) - 1
    z = z & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def gumbel_uniform(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """Python-int exact replica of the kernel's counter-based uniform (slow; tests only)."""
    m = (1 << 64) - 1
    out = []
    for i in idx.tolist():
        h = _mix64((seed * 0x9E3779B97F4A7C15 + i + 1) & m)
        out.append(((h >> 40) + 0.5) * (1.0 / 16777216.0))
    return torch.tensor(out, dtype=torch.float32)


def sample(logits, temps=None, seeds=None, vstart=0, thresh=None, check_finite=False):
    """Greedy (temp <= 0) or Gumbel-max temperature sampling; returns (ids int32, scores f32).
    `thresh[r]`: tokens whose logit / temperature is below it are excluded (top-k / top-p).
    `check_finite`: a row with an Inf / NaN logit gives id -1, score +inf."""
    lf = logits.float()
    rows, V = lf.shape
    ids, scores = [], []
    for r in range(rows):
        if check_finite and not bool(torch.isfinite(lf[r]).all()):
            ids.append(-1)
            scores.append(float("inf"))
            continue
        t = float(temps[r]) if temps is not None else 0.0
        s = lf[r]
        if t > 0:
            u = gumbel_uniform(int(seeds[r]), torch.arange(vstart, vstart + V))
            s = s * (1.0 / t)
            keep = s >= float(thresh[r]) if thresh is not None else torch.ones_like(s, dtype=torch.bool)
            s = torch.where(keep, s - torch.log(-torch.log(u)), torch.full_like(s, float("-inf")))
        i = int(torch.argmax(s))
        ids.append(i + vstart)
        scores.append(float(s[i]))
    return (torch.tensor(ids, dtype=torch.int32, device=logits.device),
            torch.tensor(scores, dtype=torch.float32, device=logits.device))


def ordered_key(s: torch.Tensor) -> torch.Tensor:
    """Order-preserving map of f32 values to u32 keys (held in int64), as in sample.hip."""
    u = s.float().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return torch.where((u & 0x80000000) != 0, (~u) & 0xFFFFFFFF, u | 0x80000000)


def unordered_key(k: int) -> float:
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return struct.unpack("<f", struct.pack("<I", u))[0]


def topkp_threshold(logits, temps, top_k, top_p, reduce_sum=None, reduce_max=None,
                    use_k: bool = True, use_p: bool = True):
    """Exact top-k / top-p thresholds on s = logit * (1 / temperature) by the same 4-pass,
    8-bit radix select as the tkp_* kernels (sample.hip), pass for pass: `reduce_sum` /
    `reduce_max` (in-place all-reduces over the TP group, or None) see the same histograms
    and row maxima, so a vocab-parallel CPU run exercises the GPU path's collective pattern.
    Returns thresh [R] f32 (-inf: row unfiltered)."""
    lf = logits.float()
    R, V = lf.shape
    inv_t = torch.where(temps > 0, 1.0 / temps.float().clamp(min=1e-30), torch.ones_like(temps.float()))
    s = lf * inv_t.view(R, 1)
    key = ordered_key(s)
    smax = (ordered_key(s.max(1).values if V else torch.full((R,), float("-inf"))) ^ 0x80000000)
    smax = torch.where(smax >= 2 ** 31, smax - 2 ** 32, smax).to(torch.int32)
    if reduce_max is not None:
        reduce_max(smax)
    mx = torch.tensor([unordered_key((int(v) & 0xFFFFFFFF) ^ 0x80000000) for v in smax.tolist()],
                      dtype=torch.float32)
    k_act = [bool(temps[r] > 0 and top_k[r] > 0) for r in range(R)]
    p_act = [bool(temps[r] > 0 and top_p[r] < 1.0) for r in range(R)]
    tk_pre, k_rem = [0] * R, [int(top_k[r]) for r in range(R)]
    tp_pre, m_above, z = [0] * R, [0.0] * R, [0.0] * R
    mass = torch.exp(s - mx.view(R, 1))
    for phase, on in ((0, use_k), (1, use_p)):
        if not on:
            continue
        for p in range(4):
            shift = 24 - 8 * p
            hist = torch.zeros(R, 512, dtype=torch.float32)
            for r in range(R):
                if not (k_act[r] if phase == 0 else p_act[r]):
                    continue
                kr = key[r]
                sel = torch.ones(V, dtype=torch.bool)
                if phase == 1 and k_act[r]:
                    sel &= kr >= tk_pre[r]
                if p > 0:
                    sel &= (kr >> (shift + 8)) == (tk_pre[r] if phase == 0 else tp_pre[r])
                d = (kr[sel] >> shift) & 255
                hist[r, :256] = torch.bincount(d, minlength=256).float()
                if phase == 1:
                    hist[r, 256:] = torch.zeros(256).index_add_(0, d, mass[r][sel])
            if reduce_sum is not None:
                reduce_sum(hist)
            for r in range(R):
                cnt, ms = hist[r, :256].tolist(), hist[r, 256:].tolist()
                if phase == 0:
                    if not k_act[r]:
                        continue
                    if p == 0 and sum(cnt) < k_rem[r]:
                        k_act[r] = False
                        continue
                    run = 0.0
                    for d in range(255, -1, -1):
                        if run < k_rem[r] <= run + cnt[d]:
                            tk_pre[r] = (tk_pre[r] << 8) | d
                            k_rem[r] -= int(run)
                            break
                        run += cnt[d]
                else:
                    if not p_act[r]:
                        continue
                    if p == 0:
                        z[r], m_above[r] = float(sum(ms)), 0.0
                    lim = float(top_p[r]) * z[r]
                    run, best, best_above = 0.0, 255, 0.0
                    for d in range(255, -1, -1):
                        if cnt[d] > 0 and m_above[r] + run <= lim:
                            best, best_above = d, run
                        run += ms[d]
                    tp_pre[r] = (tp_pre[r] << 8) | best
                    m_above[r] += best_above
    out = torch.full((R,), float("-inf"), dtype=torch.float32)
    for r in range(R):
        if k_act[r] or p_act[r]:
            kk = max(tk_pre[r] if k_act[r] else 0, tp_pre[r] if p_act[r] else 0)
            out[r] = unordered_key(kk)
    return out


def linear(x, w, bias=None, epilogue="none", out=None):
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if epilogue == "silu":
        g, u = split_gate_up(y, SILU_INTERLEAVE)
        y = F.silu(g) * u
    y = y.to(x.dtype)
    if out is None:
        return y
    out.copy_(y)
    return out


def attn_prefill(q, k, v, cu_seqlens, max_seqlen, scale, causal=True, out=None, cu_seqlens_k=None,
                 return_lse=False):
    """q [T, Hq, D], k/v [Tk, Hkv, D]; varlen sequences given by cu_seqlens (int32), keys by
    cu_seqlens_k (default: the same rows). With return_lse also returns ln sum exp(scaled
    scores) per (row, head) [T, Hq] f32, -inf where a row sees no key."""
    T, Hq, D = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    res = torch.zeros(T, Hq, D, dtype=q.dtype, device=q.device)
    lse = torch.full((T, Hq), float("-inf"), dtype=torch.float32, device=q.device)
    cu = cu_seqlens.tolist()
    cuk = cu_seqlens_k.tolist() if cu_seqlens_k is not None else cu
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        ka, kb = cuk[i], cuk[i + 1]
        if b <= a or kb <= ka:
            continue
        qs = q[a:b].float().transpose(0, 1)                       # [Hq, L, D]
        ks = k[ka:kb].float().transpose(0, 1).repeat_interleave(G, 0)
        vs = v[ka:kb].float().transpose(0, 1).repeat_interleave(G, 0)
        s = (qs @ ks.transpose(1, 2)) * scale
        if causal:
            L = b - a
            mask = torch.ones(L, kb - ka, dtype=torch.bool, device=q.device).triu(1)
            s = s.masked_fill(mask, float("-inf"))
        lse[a:b] = torch.logsumexp(s, -1).transpose(0, 1)
        p = torch.softmax(s, -1)
        res[a:b] = (p @ vs).transpose(0, 1).to(q.dtype)
    if out is not None:
        out.copy_(res)
        res = out
    return (res, lse) if return_lse else res


def attn_lse_merge_(acc_o, acc_lse, o, lse):
    """acc_lse <- log(e^acc_lse + e^lse); acc_o <- weighted mix of acc_o and o (in place)."""
    new = torch.logaddexp(acc_lse, lse)
    ok = new > float("-inf")
    wa = torch.where(ok, torch.exp(acc_lse - new), torch.zeros_like(new))
    wb = torch.where(ok, torch.exp(lse - new), torch.zeros_like(new))
    mixed = acc_o * wa.unsqueeze(-1) + o.float() * wb.unsqueeze(-1)
    acc_o.copy_(torch.where(ok.unsqueeze(-1), mixed, acc_o))
    acc_lse.copy_(torch.where(ok, new, acc_lse))
    return acc_o, acc_lse


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, max_ctx=None,
                part_tokens=None, out=None, **_):
    """q [B, Hq, D] (one token per sequence) against the paged cache."""
    B, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    res = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    for b in range(B):
        n = int(ctx_lens[b])
        nblk = (n + BS - 1) // BS
        blocks = block_tables[b, :nblk].long()
        ks = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :n].float()
        vs = v_cache[blocks].permute(1, 0, 3, 2).reshape(Hkv, nblk * BS, D)[:, :n].float()
        ks = ks.repeat_interleave(G, 0)
        vs = vs.repeat_interleave(G, 0)
        s = torch.einsum("hd,hnd->hn", q[b].float(), ks) * scale
        p = torch.softmax(s, -1)
        res[b] = torch.einsum("hn,hnd->hd", p, vs).to(q.dtype)
    if out is None:
        return res
    out.copy_(res.view(out.shape))
    return out


def attn_prefill_paged(q, k_cache, v_cache, tables, cu_q, positions, max_q, scale, out=None):
    """Chunked prefill over the paged cache: rows [cu_q[s], cu_q[s+1]) of sequence s (query
    positions `positions[row]`) attend causally to keys [0, positions[row]] of the sequence,
    read through tables[s] (the chunk's own K/V are already in the cache)."""
    T, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    res = torch.zeros(T, Hq, D, dtype=q.dtype, device=q.device)
    cu = [int(x) for x in cu_q.tolist()]
    pos = positions.long()
    for s in range(len(cu) - 1):
        a, b = cu[s], cu[s + 1]
        if b <= a:
            continue
        n = int(pos[b - 1]) + 1
        nblk = (n + BS - 1) // BS
        blocks = tables[s, :nblk].long()
        ks = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :n].float().repeat_interleave(G, 0)
        vs = v_cache[blocks].permute(1, 0, 3, 2).reshape(Hkv, nblk * BS, D)[:, :n].float().repeat_interleave(G, 0)
        sc = torch.einsum("thd,hnd->htn", q[a:b].float(), ks) * scale
        mask = torch.arange(n, device=q.device)[None, :] > pos[a:b, None]
        sc = sc.masked_fill(mask[None], float("-inf"))
        res[a:b] = torch.einsum("htn,hnd->thd", torch.softmax(sc, -1), vs).to(q.dtype)
    if out is None:
        return res
    out.copy_(res)
    return out


# ---------------------------------------------------------------------------------------
# Deterministic init and MoE gating
# ---------------------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _fmix32(h):
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def init_hash(out, grow0, gcol0, gcols, seed, amp):
    """Value of global element (r, c) = amp * (2u - 1), u = hash(seed, r*gcols + c)."""
    rows, cols = out.shape
    r = torch.arange(rows, dtype=torch.int64).unsqueeze(1) + grow0
    c = torch.arange(cols, dtype=torch.int64).unsqueeze(0) + gcol0
    idx = (r * gcols + c) & _M32
    h = _fmix32((idx * 0x9E3779B1 + seed) & _M32)
    u = (h >> 8).to(torch.float32) * (1.0 / 16777216.0) + (0.5 / 16777216.0)
    out.copy_((amp * (2.0 * u - 1.0)).to(out.dtype))
    return out


def moe_route(x, wr, top_k):
    """-> (gates [T, E] f32 dense, topk_ids [T, k] int32, topk_w [T, k] f32); Mixtral
    semantics: softmax over all experts, top-k, renormalise over the selected."""
    logits = x.float() @ wr.float().t()
    p = torch.softmax(logits, -1)
    w, ids = torch.topk(p, top_k, -1)
    w = w / w.sum(-1, keepdim=True)
    gates = torch.zeros_like(p).scatter_(1, ids, w)
    return gates, ids.to(torch.int32), w


def moe_gate_scale(h, gates, e0, num_local):
    T = h.shape[0]
    F = h.shape[1] // num_local
    g = gates[:, e0:e0 + num_local].to(torch.float32)
    v = h.float().view(T, num_local, F) * g.unsqueeze(-1)
    h.copy_(v.view(T, num_local * F).to(h.dtype))
    return h


def moe_sparse_ffn(x, topk_ids, topk_w, gu_w, down_w, e0: int, num_local: int, ffn: int):
    """Token-routed expert FFN over the local experts (SwiGLU, gate/up interleaved rows):
    out[t] = sum_j w[t, j] * down_e(silu(g_e x_t) * u_e x_t) for j with local e = ids[t, j]."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    ids = topk_ids.long() - e0
    for el in range(num_local):
        hit = (ids == el)
        tok = hit.any(-1).nonzero().flatten()
        if tok.numel() == 0:
            continue
        w_e = (topk_w * hit).sum(-1)[tok]
        gu = gu_w[el * 2 * ffn:(el + 1) * 2 * ffn]
        h = linear(x[tok], gu, epilogue="silu")
        y = linear(h, down_w[:, el * ffn:(el + 1) * ffn].contiguous())
        out[tok] += w_e.unsqueeze(-1).float() * y.float()
    return out.to(x.dtype)


def ep_pack(x, ids, w, slots, experts_per_rank: int, ep: int, cap: int):
    """Fixed-capacity EP dispatch (reference of ep_pack_kernel): token t goes once to every
    rank d owning one of its experts, at row d * cap + (number of earlier tokens bound for d).
    Returns send [ep*cap, H], meta [ep*cap, 2k] f32 (expert ids local to the row's rank as
    int32 bits, -1 otherwise; gate weights), slot [T, ep] int32 (-1: not sent)."""
    T, H = x.shape
    k = ids.shape[1]
    idl = ids.long()
    if slots is not None:
        idl = idl.masked_fill((slots < 0).unsqueeze(1), -1)
    dest = torch.where(idl >= 0, torch.div(idl.clamp(min=0), experts_per_rank, rounding_mode="floor"), ep)
    hit = torch.zeros(T, ep + 1, dtype=torch.int64)
    if T:
        hit.scatter_(1, dest, 1)
    hit = hit[:, :ep]
    pos = torch.cumsum(hit, 0) - hit
    slot = torch.where(hit > 0, torch.arange(ep) * cap + pos, -1)
    send = torch.zeros(ep * cap, H, dtype=x.dtype)
    mid = torch.full((ep * cap, k), -1, dtype=torch.int32)
    mw = torch.zeros(ep * cap, k, dtype=torch.float32)
    for t in range(T):
        for d in range(ep):
            r = int(slot[t, d])
            if r < 0:
                continue
            send[r] = x[t]
            mine = dest[t] == d
            mid[r] = torch.where(mine, idl[t], -1).to(torch.int32)
            mw[r] = torch.where(mine, w[t].float(), 0.0)
    meta = torch.cat([mid.view(torch.float32), mw], 1)
    return send, meta, slot.to(torch.int32)


def ep_combine(back, slot):
    """out[t] = sum of back[slot[t, d]] over the ranks d token t was sent to (f32 sum)."""
    T, ep = slot.shape
    if T == 0:
        return back.new_zeros(0, back.shape[1])
    ext = torch.cat([back.float(), back.new_zeros(1, back.shape[1]).float()])
    idx = torch.where(slot >= 0, slot.long(), back.shape[0])
    return ext.index_select(0, idx.view(-1)).view(T, ep, -1).sum(1).to(back.dtype)
