"""C++ host runtime: KV page manager, scheduler policy, pipeline cut DP (vs brute force)."""
import itertools

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from butterfly_amd._native_loader import native

N = native()


def test_kv_manager_alloc_append_free_fork():
    kv = N.KVBlockManager(8, 4)
    slots = kv.allocate(1, 6)
    assert len(slots) == 6 and kv.num_free == 6
    assert slots[:4] == [slots[0] + i for i in range(4)]
    s, src, dst = kv.append_slot(1)            # 7th token, same page
    assert src == -1 and kv.length(1) == 7
    kv.append_slot(1)
    s, src, dst = kv.append_slot(1)            # 9th token -> new page
    assert kv.num_free == 5 and src == -1
    kv.fork(1, 2)
    s, src, dst = kv.append_slot(2)            # shared last page -> copy on write
    assert src >= 0 and dst >= 0 and src != dst
    tables = np.zeros((2, 8), dtype=np.int32)
    ctx = np.zeros(2, dtype=np.int32)
    kv.fill_decode_tables([1, 2], tables, ctx)
    assert list(ctx) == [9, 10]
    kv.free(1)
    kv.free(2)
    assert kv.num_free == 8
    with pytest.raises(RuntimeError):
        kv.allocate(3, 33)


def test_scheduler_prefill_then_decode_and_preempt():
    kv = N.KVBlockManager(4, 4)                # 16 token slots
    s = N.Scheduler(kv, 8, 64)
    s.add(1, 6, 10)
    s.add(2, 5, 10)
    p = s.schedule()
    assert p.kind == 1 and list(p.seq_ids) == [1, 2] and [len(x) for x in p.prefill_slots] == [6, 5]
    s.on_token(1)
    s.on_token(2)
    for _ in range(2):
        p = s.schedule()
        assert p.kind == 2
        s.on_token(1)
        s.on_token(2)
    # 4 pages: seq1 8 tok (2 pages) seq2 7 tok (2 pages); next append needs a page -> preempt newest
    p = s.schedule()
    assert p.kind == 2 and list(p.preempted) == [2] and list(p.seq_ids) == [1]
    assert s.num_waiting == 1


def _brute(t, P, cap, mem):
    L = len(t)
    best = None
    for cuts in itertools.combinations(range(1, L), P - 1):
        c = (0,) + cuts + (L,)
        if any(sum(mem[c[i]:c[i + 1]]) > cap for i in range(P)):
            continue
        v = max(sum(t[c[i]:c[i + 1]]) for i in range(P))
        if best is None or v < best:
            best = v
    return best


@settings(max_examples=60, deadline=None)
@given(st.lists(st.integers(1, 20), min_size=2, max_size=9), st.integers(1, 4), st.integers(10, 200))
def test_pipeline_cuts_optimal(ts, P, cap):
    P = min(P, len(ts))
    t = [float(x) for x in ts]
    m = [float(x) for x in ts]
    cuts = N.pipeline_cuts(t, m, P, 0.0, 0.0, 0.0, 0.0, 0.0, float(cap))
    ref = _brute(t, P, cap, m)
    if ref is None:
        assert cuts == []
        return
    assert cuts[0] == 0 and cuts[-1] == len(t) and len(cuts) == P + 1
    assert all(cuts[i] < cuts[i + 1] for i in range(P))
    got = max(sum(t[cuts[i]:cuts[i + 1]]) for i in range(P))
    assert got == ref
