"""Device top-k / top-p (engine/sampler.py): one exact radix-selected threshold per row on
logit * (1 / temperature), Gumbel-max over the kept set. Checked against an exact sort-based
reference of the truncated set (including 128k-vocab, high-entropy rows whose nucleus holds
thousands of tokens), across TP splits of the vocabulary (loopback ranks), and end to end."""
import pytest
import torch

from butterfly_amd.engine.sampler import Sampler, SamplingParams
from butterfly_amd.parallel.fake import FakeWorld
from butterfly_amd.parallel.mesh import Mesh


def exact_keep(row: torch.Tensor, temp: float, top_k: int, top_p: float) -> torch.Tensor:
    """The kept token set by sorting (top-k first, then the nucleus of the renormalised rest)."""
    s = row.float() * (1.0 / torch.tensor(temp, dtype=torch.float32))   # the kernels' f32 scaling
    order = torch.argsort(s, descending=True)
    sv = s[order]
    n = len(sv) if top_k <= 0 else min(top_k, len(sv))
    keep = torch.zeros(len(s), dtype=torch.bool)
    sv = sv[:n]
    pr = torch.softmax(sv, 0)
    before = pr.cumsum(0) - pr
    m = int((before <= top_p).sum()) if top_p < 1.0 else n
    keep[order[:max(1, m)]] = True
    return keep


def value_threshold(row: torch.Tensor, temp: float, top_k: int, top_p: float) -> float:
    """Tie-aware exact threshold (a value filter keeps whole tie groups): top-k keeps every
    token >= the k-th largest value; top-p then keeps each value whose strictly larger tokens
    hold <= p of the (top-k renormalised) mass."""
    s = row.float() * (1.0 / torch.tensor(temp, dtype=torch.float32))
    sv = torch.sort(s, descending=True).values.double()
    t = float("-inf")
    if top_k > 0:
        t = float(sv[min(top_k, len(sv)) - 1])
        sv = sv[sv >= t]
    if top_p < 1.0:
        vals, counts = torch.unique_consecutive(sv, return_counts=True)
        mass = torch.exp(vals - vals[0]) * counts
        above = torch.cumsum(mass, 0) - mass               # mass strictly above each value
        ok = above <= top_p * mass.sum()
        t = max(t, float(vals[ok].min()))
    return t


CASES = [SamplingParams(temperature=0.8, top_k=5), SamplingParams(temperature=1.0, top_p=0.3),
         SamplingParams(temperature=0.7, top_k=40, top_p=0.5), SamplingParams(temperature=1.3, top_p=0.9),
         SamplingParams(temperature=1.0, top_k=1)]


def test_thresholds_match_exact_sets():
    torch.manual_seed(0)
    V = 700
    logits = torch.randn(len(CASES), V) * 3
    smp = Sampler(None, V, 0, 1)
    temps = torch.tensor([p.temperature for p in CASES])
    thr = smp.thresholds(logits, temps, CASES)
    for r, p in enumerate(CASES):
        got = (logits[r].float() * (1.0 / torch.tensor(p.temperature))) >= thr[r]
        assert torch.equal(got, exact_keep(logits[r], p.temperature, p.top_k, p.top_p)), r


@pytest.mark.parametrize("tp", [2, 4])
def test_thresholds_are_tp_invariant(tp):
    """Vocab-parallel shards (loopback TP ranks) agree on the same thresholds as one rank."""
    torch.manual_seed(1)
    V = 512
    logits = torch.randn(len(CASES), V) * 2
    temps = torch.tensor([p.temperature for p in CASES])
    ref = Sampler(None, V, 0, 1).thresholds(logits, temps, CASES)
    world = FakeWorld(Mesh(tp=tp))

    def body(rank, comm):
        Vl = V // tp
        smp = Sampler(comm, V, rank * Vl, tp)
        return smp.thresholds(logits[:, rank * Vl:(rank + 1) * Vl], temps, CASES)

    for thr in world.run(body):
        torch.testing.assert_close(thr, ref)


def test_filtered_sampling_stays_in_set_and_is_tp_invariant():
    torch.manual_seed(2)
    V = 256
    logits = torch.randn(len(CASES), V) * 2
    seeds = torch.arange(len(CASES), dtype=torch.int64) * 7 + 3
    one = Sampler(None, V, 0, 1).sample(logits, torch.tensor([p.temperature for p in CASES]), seeds, CASES)
    for r, p in enumerate(CASES):
        assert exact_keep(logits[r], p.temperature, p.top_k, p.top_p)[int(one[r])]
    world = FakeWorld(Mesh(tp=2))

    def body(rank, comm):
        smp = Sampler(comm, V, rank * V // 2, 2)
        return smp.sample(logits[:, rank * V // 2:(rank + 1) * V // 2],
                          torch.tensor([p.temperature for p in CASES]), seeds, CASES)

    for ids in world.run(body):
        assert torch.equal(ids, one)


def test_wide_nucleus_128k_vocab_is_exact():
    """High-entropy rows over a Llama-3-sized vocabulary: the nucleus holds far more than the
    1,024 candidates the previous top-C scheme could see; the radix select stays exact."""
    torch.manual_seed(3)
    V = 128256
    params = [SamplingParams(temperature=1.0, top_p=0.9), SamplingParams(temperature=1.5, top_k=5000, top_p=0.95),
              SamplingParams(temperature=0.9, top_k=3000), SamplingParams(temperature=1.0, top_p=0.5)]
    logits = (torch.randn(len(params), V) * 0.5).to(torch.bfloat16)
    temps = torch.tensor([p.temperature for p in params])
    thr = Sampler(None, V, 0, 1).thresholds(logits, temps, params)
    for r, p in enumerate(params):
        keep = exact_keep(logits[r], p.temperature, p.top_k, p.top_p)
        got = (logits[r].float() * (1.0 / torch.tensor(p.temperature))) >= thr[r]
        assert int(keep.sum()) > 1024
        # bf16 logits tie: a value threshold keeps whole tie groups (value_threshold)
        assert float(thr[r]) == value_threshold(logits[r], p.temperature, p.top_k, p.top_p), r


@pytest.mark.parametrize("tp", [2, 4])
def test_narrow_filters_with_empty_shards(tp):
    """top_k=1 / tiny top_p leave most vocab shards with no candidate: the merged id must be
    the single-rank id (an empty shard scores -inf, never NaN / id -1)."""
    torch.manual_seed(4)
    V = 1024
    params = [SamplingParams(temperature=1.0, top_k=1), SamplingParams(temperature=0.8, top_p=0.01),
              SamplingParams(temperature=1.2, top_k=2, top_p=0.5)]
    logits = torch.randn(len(params), V) * 4
    temps = torch.tensor([p.temperature for p in params])
    seeds = torch.tensor([11, 12, 13], dtype=torch.int64)
    one = Sampler(None, V, 0, 1).sample(logits, temps, seeds, params, check_finite=True)
    assert int(one[0]) == int(logits[0].argmax())
    world = FakeWorld(Mesh(tp=tp))

    def body(rank, comm):
        Vl = V // tp
        return Sampler(comm, V, rank * Vl, tp).sample(logits[:, rank * Vl:(rank + 1) * Vl], temps, seeds, params,
                                                      check_finite=True)

    for ids in world.run(body):
        assert torch.equal(ids, one)
