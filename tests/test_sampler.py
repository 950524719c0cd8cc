"""Device top-k / top-p (engine/sampler.py): one threshold per row on logit / temperature,
Gumbel-max over the kept set. Checked against an exact sort-based reference of the truncated
set, across TP splits of the vocabulary (loopback ranks), and end to end."""
import pytest
import torch

from butterfly_amd.engine.sampler import Sampler, SamplingParams
from butterfly_amd.parallel.fake import FakeWorld
from butterfly_amd.parallel.mesh import Mesh


def exact_keep(row: torch.Tensor, temp: float, top_k: int, top_p: float) -> torch.Tensor:
    """The kept token set by sorting (top-k first, then the nucleus of the renormalised rest)."""
    s = row.float() / temp
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
        got = (logits[r].float() / p.temperature) >= thr[r]
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
