"""Distributed correctness on CPU/gloo: every parallel layout of the engine generates exactly
the tokens of the single-process engine with the same (partition-independent) weights.

Covers the BASELINE.json CPU plumbing config (GPT-2 small, 2-stage layer split, world 2) and
TP, PP, TP x PP, DP and expert parallelism (Mixtral) on small configs."""
import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams
from butterfly_amd.parallel.mesh import Mesh

from .dist_utils import run_world

PROMPTS = [[3, 14, 15, 92, 65], [35, 89, 79, 32, 38, 46, 26], [43], [38, 32, 79, 50, 28, 84]]


def _engine(preset, mesh=Mesh(), comm=None, max_tokens=6):
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    return LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")


def _single(preset, prompts, max_tokens=6):
    return _engine(preset).generate(prompts, SamplingParams(max_tokens=max_tokens, ignore_eos=True))


def _dist_generate(rank, world, preset, mesh_kw, prompts_per_dp, max_tokens):
    from butterfly_amd.parallel.comm import Communicator

    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh)
    eng = _engine(preset, mesh, comm)
    prompts = prompts_per_dp[mesh.coord(rank).dp]
    return eng.generate(prompts, SamplingParams(max_tokens=max_tokens, ignore_eos=True))


@pytest.mark.parametrize("preset,mesh_kw,world", [
    ("gpt2-small", dict(pp=2), 2),          # BASELINE config 1: GPT-2 small 2-stage split, gloo
    ("llama-tiny", dict(tp=2), 2),
    ("llama-tiny", dict(pp=2), 2),
    ("gpt2-tiny", dict(tp=2), 2),
    ("mixtral-tiny", dict(tp=2), 2),
    ("llama-tiny", dict(tp=2, pp=2), 4),
])
def test_model_parallel_matches_single(preset, mesh_kw, world):
    n = 3 if preset == "gpt2-small" else 6
    prompts = PROMPTS[:2] if preset == "gpt2-small" else PROMPTS
    ref = _single(preset, prompts, n)
    outs = run_world(_dist_generate, world, preset, mesh_kw, [prompts], n)
    for o in outs:
        assert o == ref


def _mixed_generate(rank, world, preset, mesh_kw, max_batch, async_pp, async_decode=False):
    """Requests of different lengths, more than the batch holds (admission while the pipeline
    runs), one request added mid-run; per-request outputs."""
    import os

    from butterfly_amd.parallel.comm import Communicator

    saved = os.environ.get("BFLY_PP_ASYNC")
    os.environ["BFLY_PP_ASYNC"] = "1" if async_pp else "0"
    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh) if world > 1 else None
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=max_batch, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5,
                        async_decode=async_decode)
    try:
        eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")   # reads the flag
        assert eng.async_pp == (async_pp and (mesh.pp > 1 or async_decode))
    finally:   # the single-process reference runs in the test process: do not leak the flag
        if saved is None:
            os.environ.pop("BFLY_PP_ASYNC", None)
        else:
            os.environ["BFLY_PP_ASYNC"] = saved
    rids = [eng.add_request(p, SamplingParams(max_tokens=3 + 2 * i, ignore_eos=True))
            for i, p in enumerate(PROMPTS + PROMPTS[:2])]
    for _ in range(5):
        eng.step()
    rids.append(eng.add_request([7, 7, 7], SamplingParams(max_tokens=4, ignore_eos=True)))
    while eng.has_unfinished():
        eng.step()
    return [eng.requests[r].output for r in rids]


def test_async_decode_single_stage_matches_single():
    """EngineConfig.async_decode (pp == 1): step k+1 is scheduled and its input ids gathered on
    the device before step k's token values reach the host; same tokens, stop handling and
    admission as the synchronous engine."""
    assert _mixed_generate(0, 1, "llama-tiny", {}, 4, True, async_decode=True) == \
        _mixed_generate(0, 1, "llama-tiny", {}, 4, False)


@pytest.mark.parametrize("preset,mesh_kw,world", [
    ("llama-tiny", dict(tp=2), 2),
])
def test_async_decode_tp_matches_single(preset, mesh_kw, world):
    ref = _mixed_generate(0, 1, preset, {}, 4, False)
    for o in run_world(_mixed_generate, world, preset, mesh_kw, 4, True, True):
        assert o == ref


@pytest.mark.parametrize("preset,mesh_kw,world", [
    ("llama-tiny", dict(pp=2), 2),
    ("llama-small", dict(pp=4), 4),
    ("llama-tiny", dict(tp=2, pp=2), 4),
])
def test_async_pipeline_matches_single(preset, mesh_kw, world):
    ref = _mixed_generate(0, 1, preset, {}, 4, False)
    outs = run_world(_mixed_generate, world, preset, mesh_kw, 4, True)
    for o in outs:
        assert o == ref
    # and the synchronous microbatched pipeline gives the same tokens
    if world == 2:
        assert run_world(_mixed_generate, world, preset, mesh_kw, 4, False)[0] == ref


LONG = [[(7 * i + 3) % 97 + 1 for i in range(40)], [(5 * i + 1) % 89 + 1 for i in range(23)]]


def _chunked_generate(rank, world, preset, mesh_kw, async_pp, shared_prefix=False, kv_tokens=2048, prompts=None,
                      max_new=4, max_batch=4):
    """Prompts longer than the step's token budget (prefilled in chunks over several steps /
    ticks, decode rows riding along), more requests than the batch holds, a request added
    mid-run; with `shared_prefix` every prompt starts with the same 64 tokens (prefix cache);
    with a small `kv_tokens` the cache forces preemption and recompute."""
    import os

    from butterfly_amd.parallel.comm import Communicator

    saved = os.environ.get("BFLY_PP_ASYNC")
    os.environ["BFLY_PP_ASYNC"] = "1" if async_pp else "0"
    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh) if world > 1 else None
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=max_batch, max_seq_len=160, kv_cache_tokens=kv_tokens, max_prefill_tokens=24,
                        use_graphs=False, seed=5, async_decode=async_pp, mixed_prefill=True, prefix_caching=True)
    try:
        eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")
        assert eng.mixed and eng.async_pp == async_pp
    finally:
        if saved is None:
            os.environ.pop("BFLY_PP_ASYNC", None)
        else:
            os.environ["BFLY_PP_ASYNC"] = saved
    head = [(11 * i) % 83 + 2 for i in range(64)] if shared_prefix else []
    prompts = [head + p for p in (prompts or LONG + PROMPTS)]
    rids = [eng.add_request(p, SamplingParams(max_tokens=max_new + i, ignore_eos=True)) for i, p in enumerate(prompts)]
    kinds = set()
    for _ in range(4):
        kinds.add(eng.step().kind)
    rids.append(eng.add_request(head + LONG[0][:30], SamplingParams(max_tokens=5, ignore_eos=True)))
    while eng.has_unfinished():
        kinds.add(eng.step().kind)
    hits = eng.scheduler.prefix_hit_tokens
    pre = eng.metrics.counters.get("preempted_sequences", 0) if hasattr(eng.metrics, "counters") else 0
    return [eng.requests[r].output for r in rids], sorted(kinds), hits, pre


@pytest.mark.parametrize("preset,mesh_kw,world,mb", [
    ("llama-tiny", {}, 1, 4),
    ("llama-tiny", dict(pp=2), 2, 4),
    ("llama-tiny", dict(tp=2), 2, 4),
    ("llama-tiny", dict(tp=2, pp=2), 4, 4),
    ("llama-small", dict(pp=4), 4, 8),      # 4 groups of 2: a decode row beside each chunk
])
@pytest.mark.parametrize("shared_prefix", [False, True])
def test_async_mixed_chunked_prefill_matches_sync(preset, mesh_kw, world, mb, shared_prefix):
    """Mixed plans (decode rows + prompt chunks) in the asynchronous pipeline: chunked prompts
    over several ticks, prefix-cache hits, PP stages: the tokens of the synchronous
    single-process engine."""
    ref, ref_kinds, _, _ = _chunked_generate(0, 1, preset, {}, False, shared_prefix, max_batch=mb)
    assert "mixed" in ref_kinds
    outs = (run_world(_chunked_generate, world, preset, mesh_kw, True, shared_prefix, 2048, None, 4, mb) if world > 1
            else [_chunked_generate(0, 1, preset, {}, True, shared_prefix, max_batch=mb)])
    for o, kinds, hits, _ in outs:
        assert o == ref
        assert "mixed" in kinds
        if shared_prefix:
            assert hits > 0


def test_async_mixed_preemption_recompute_matches_sync():
    """A KV cache too small for every running sequence: preempted sequences are re-prefilled
    (prompt + tokens generated so far) in later chunks, including the token sampled by the
    plan right before (its value read from the pinned copy, not yet applied)."""
    prompts = [[(3 * i + j) % 90 + 1 for i in range(30)] for j in range(4)]
    ref, _, _, pre = _chunked_generate(0, 1, "llama-tiny", {}, False, kv_tokens=160, prompts=prompts, max_new=12)
    got, _, _, pre_async = _chunked_generate(0, 1, "llama-tiny", {}, True, kv_tokens=160, prompts=prompts, max_new=12)
    assert pre > 0 and pre_async > 0, "the configuration must preempt"
    assert got == ref


def test_data_parallel_replicas():
    halves = [PROMPTS[:2], PROMPTS[2:]]
    outs = run_world(_dist_generate, 2, "llama-tiny", dict(dp=2), halves, 6)
    assert outs[0] == _single("llama-tiny", halves[0])
    assert outs[1] == _single("llama-tiny", halves[1])


def test_expert_parallel_mixtral():
    # DP-attention + EP experts: each rank serves its own prompts, experts split 2 ways;
    # the second replica gets fewer requests (exercises padding and idle-rank steps).
    halves = [PROMPTS[:3], PROMPTS[3:]]
    outs = run_world(_dist_generate, 2, "mixtral-tiny", dict(dp=2, ep=2), halves, 6)
    assert outs[0] == _single("mixtral-tiny", halves[0])
    assert outs[1] == _single("mixtral-tiny", halves[1])


def _ep_async_generate(rank, world, mesh_kw, async_pp):
    """Expert-parallel replicas with uneven loads (replica r gets r + 1 requests, one more added
    mid-run on replica 0 only): idle ranks must keep joining their peers' MoE exchanges."""
    import os

    from butterfly_amd.parallel.comm import Communicator

    saved = os.environ.get("BFLY_PP_ASYNC")
    os.environ["BFLY_PP_ASYNC"] = "1" if async_pp else "0"
    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh)
    cfg = ModelConfig.from_preset("mixtral-tiny")
    ecfg = EngineConfig(max_batch=4, max_seq_len=96, kv_cache_tokens=1024, use_graphs=False, seed=5)
    try:
        eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")
        assert eng.async_pp == async_pp
    finally:
        if saved is None:
            os.environ.pop("BFLY_PP_ASYNC", None)
        else:
            os.environ["BFLY_PP_ASYNC"] = saved
    dp = mesh.coord(rank).dp
    mine = [PROMPTS[(dp + i) % len(PROMPTS)] for i in range(dp + 1)]
    rids = [eng.add_request(p, SamplingParams(max_tokens=3 + i + dp, ignore_eos=True)) for i, p in enumerate(mine)]
    for _ in range(3):
        eng.step()
    if dp == 0:
        rids.append(eng.add_request([9, 8, 7], SamplingParams(max_tokens=5, ignore_eos=True)))
    while eng.has_unfinished_global():
        eng.step()
    return [eng.requests[r].output for r in rids]


def test_expert_parallel_with_pipeline_stages():
    """EP x PP: Mixtral experts split over 2 replicas, each replica a 2-stage
    pipeline (4 ranks); each stage's MoE layers exchange tokens with the other replica's same
    stage. Uneven loads (idle plans travel the pipeline): every replica's tokens equal the
    synchronous EP engine's (= single process)."""
    ref = run_world(_ep_async_generate, 2, dict(dp=2, ep=2), False)
    got = run_world(_ep_async_generate, 4, dict(dp=2, ep=2, pp=2), True)
    mesh = Mesh(dp=2, ep=2, pp=2)
    for r in range(4):
        assert got[r] == ref[mesh.coord(r).dp], r


@pytest.mark.parametrize("mesh_kw,world", [(dict(dp=2, ep=2), 2), (dict(dp=4, ep=4), 4)])
def test_expert_parallel_async_matches_sync(mesh_kw, world):
    """EP layouts on the asynchronous engine (host agreement over the control plane, token
    values one step late) give every replica the tokens of the synchronous EP engine."""
    ref = run_world(_ep_async_generate, world, mesh_kw, False)
    got = run_world(_ep_async_generate, world, mesh_kw, True)
    assert got == ref


def _ep_mixed_generate(rank, world, mesh_kw, async_pp, shared_prefix, long_len=0):
    """Expert-parallel replicas on the mixed scheduler: long prompts prefilled in chunks
    beside decode rows (token budget 24), uneven loads per replica (one replica gets the long
    prompt, the other only short ones), prefix caching; `mesh_kw` {} = the single-process
    reference serving replica `rank`'s requests."""
    import os

    from butterfly_amd.parallel.comm import Communicator

    saved = os.environ.get("BFLY_PP_ASYNC")
    os.environ["BFLY_PP_ASYNC"] = "1" if async_pp else "0"
    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh) if mesh.world_size > 1 else None
    cfg = ModelConfig.from_preset("mixtral-tiny")
    ecfg = EngineConfig(max_batch=4, max_seq_len=max(160, long_len + 96), kv_cache_tokens=4096,
                        max_prefill_tokens=24, use_graphs=False, seed=5, async_decode=async_pp,
                        mixed_prefill=True, prefix_caching=True)
    try:
        eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")
        assert eng.mixed and eng.async_pp == async_pp
    finally:
        if saved is None:
            os.environ.pop("BFLY_PP_ASYNC", None)
        else:
            os.environ["BFLY_PP_ASYNC"] = saved
    dp = rank if mesh.world_size == 1 else mesh.coord(rank).dp
    head = [(11 * i) % 83 + 2 for i in range(64)] if shared_prefix else []
    longp = [[(13 * i + 5) % 91 + 1 for i in range(long_len)]] if long_len else []
    mine = (longp + LONG) if dp == 0 else PROMPTS[: 1 + dp]
    rids = [eng.add_request(head + p, SamplingParams(max_tokens=3 + i, ignore_eos=True)) for i, p in enumerate(mine)]
    kinds = set()
    for _ in range(3):
        kinds.add(eng.step().kind)
    if dp == 0:
        rids.append(eng.add_request(head + LONG[1][:20], SamplingParams(max_tokens=4, ignore_eos=True)))
    step = eng.has_unfinished_global if mesh.world_size > 1 else eng.has_unfinished
    while step():
        kinds.add(eng.step().kind)
    return [eng.requests[r].output for r in rids], sorted(kinds), eng.scheduler.prefix_hit_tokens


@pytest.mark.parametrize("mesh_kw,world,async_pp", [(dict(dp=2, ep=2), 2, True), (dict(dp=2, ep=2), 2, False),
                                                   (dict(dp=4, ep=4), 4, True), (dict(dp=4, ep=4), 4, False),
                                                   (dict(dp=2, ep=2, pp=2), 4, True)])
@pytest.mark.parametrize("shared_prefix", [False, True])
def test_expert_parallel_mixed_chunked_prefill(mesh_kw, world, async_pp, shared_prefix):
    """expert-parallel layouts run mixed plans (prompt chunks beside decode
    rows, prefix caching) on the asynchronous and the synchronous engine; every replica's
    tokens equal the single-process engine's for the same requests."""
    long_len = 300 if world == 2 else 0
    got = run_world(_ep_mixed_generate, world, mesh_kw, async_pp, shared_prefix, long_len)
    mesh = Mesh(**mesh_kw)
    for r in range(world):
        dp = mesh.coord(r).dp
        want, want_kinds, _ = _ep_mixed_generate(dp, 1, {}, False, shared_prefix, long_len)
        out, kinds, hits = got[r]
        assert out == want, r
        if dp == 0 and mesh.coord(r).pp == mesh.pp - 1:
            assert "mixed" in want_kinds and "mixed" in kinds
            if shared_prefix:
                assert hits > 0


def _probe_worker(rank, world):
    import torch

    from butterfly_amd.parallel.probe import ar_policy, probe_comm, summarize

    tab = probe_comm(world, device=torch.device("cpu"), iters=2, butterfly=True)
    return tab, ar_policy(tab), summarize(tab)


def test_comm_probe_plumbing_gloo():
    """The start-up probe (parallel/probe.py) on 4 gloo ranks: groups of 2 and 4 timed at once,
    send/recv pairs and all-to-all; every rank ends with the identical (max-reduced) table,
    which the cost model can consume."""
    from butterfly_amd.config import ModelConfig
    from butterfly_amd.partition.costmodel import CostModel
    from butterfly_amd.partition.hw import MI355X

    res = run_world(_probe_worker, 4)
    tabs = [r[0] for r in res]
    assert all(t["all_reduce"] == tabs[0]["all_reduce"] and t["p2p"] == tabs[0]["p2p"] for t in tabs)
    ar = tabs[0]["all_reduce"]["rccl"]
    assert sorted(ar) == [2, 4] and all(len(v) == 6 for v in ar.values())
    assert len(tabs[0]["p2p"]) == 3 and 4 in tabs[0]["all_to_all"]
    assert res[0][1][4]["ipc_max"] == 0            # no IPC kernel on CPU: RCCL-only policy
    bf = tabs[0]["all_reduce"]["butterfly"]         # the butterfly is timed on every pow2 group
    assert sorted(bf) == [2, 4] and all(len(v) == 6 for v in bf.values())
    for n in (2, 4):
        rng = res[0][1][n]["butterfly"]
        assert rng is None or (rng[0] <= rng[1] and all(r[1][n]["butterfly"] == rng for r in res))
    cm = CostModel(ModelConfig.from_preset("llama3-8b"), MI355X.with_comm_table(dict(tabs[0], policy=res[0][1])))
    assert cm.allreduce(1 << 20, 4) > 0 and cm.p2p(1 << 20) > 0


def _stop_generate(rank, world, stop_tok):
    """Async pipeline with a stop token that fires while the stopped sequence's next plan is
    already in flight (values are applied one tick late)."""
    from butterfly_amd.parallel.comm import Communicator

    mesh = Mesh(pp=2) if world > 1 else Mesh()
    comm = Communicator.from_mesh(mesh) if world > 1 else None
    cfg = ModelConfig.from_preset("llama-tiny")
    ecfg = EngineConfig(max_batch=4, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")
    params = [SamplingParams(max_tokens=12, stop_token_ids=[stop_tok]), SamplingParams(max_tokens=12)]
    rids = [eng.add_request(p, params[i % 2]) for i, p in enumerate(PROMPTS)]
    while eng.has_unfinished():
        eng.step()
    kv_free = eng.kv.manager.num_free
    return [eng.requests[r].output for r in rids], [eng.requests[r].finish_reason for r in rids], kv_free


def test_async_pipeline_stop_token_matches_single():
    """Lagged token values (engine._pp_tick): a sequence that emits its stop token is cut at
    exactly the same place as in a single-process run, the extra in-flight token is dropped,
    and every KV block comes back."""
    free_ref = _stop_generate(0, 1, 0)
    # pick a stop token the first prompt actually produces mid-sequence
    stop_tok = free_ref[0][0][4]
    ref_out, ref_reason, ref_free = _stop_generate(0, 1, stop_tok)
    outs = run_world(_stop_generate, 2, stop_tok)
    assert ref_reason[0] == "stop"
    for out, reason, free in outs:
        assert out == ref_out and reason == ref_reason and free == ref_free


def _sp_generate(rank, world, preset, mesh_kw, prompts, max_tokens):
    import os

    os.environ["BFLY_SEQ_PARALLEL"] = "1"          # spawned rank: the flag stays in this process
    os.environ["BFLY_SEQ_PARALLEL_MIN_TOKENS"] = "1"
    from butterfly_amd.parallel.comm import Communicator

    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh)
    eng = _engine(preset, mesh, comm)
    assert eng.model.seq_parallel
    sent = []
    orig = comm.reduce_scatter
    comm.reduce_scatter = lambda t, group="ep", out=None: (sent.append(group), orig(t, group, out))[1]
    outs = eng.generate(prompts, SamplingParams(max_tokens=max_tokens, ignore_eos=True))
    return outs, sent.count("tp")


@pytest.mark.parametrize("preset,mesh_kw,world", [
    ("llama-tiny", dict(tp=2), 2),
    ("gpt2-tiny", dict(tp=2), 2),          # learned positions, LayerNorm, biases
    ("mixtral-tiny", dict(tp=2), 2),
    ("llama-tiny", dict(tp=2, pp=2), 4),
])
def test_sequence_parallel_prefill_matches_single(preset, mesh_kw, world):
    """Megatron sequence parallelism on TP prefill steps (reduce-scatter into token shards, norms
    on the shard, all-gather before the column-parallel GEMMs; T = 19 is not a multiple of tp,
    so the padding rows are exercised) generates exactly the single-process tokens."""
    ref = _single(preset, PROMPTS, 5)
    outs = run_world(_sp_generate, world, preset, mesh_kw, PROMPTS, 5)
    for toks, n_rs in outs:
        assert toks == ref
        assert n_rs > 0          # the SP path really ran


def test_mixed_step_splits_continuations_from_fresh_prompts(monkeypatch):
    """A mixed step whose leading chunks continue cached prompts and whose remaining chunks are
    fresh runs the paged pass on the continuations only and flash attention on the fresh
    prompts (ForwardBatch.split_seqs); the tokens equal the all-paged path's."""
    from butterfly_amd.engine.model_runner import ModelRunner

    orig = ModelRunner.mixed_batch
    seen = []

    def counting(self, plan, tokens_of):
        fb, sample = orig(self, plan, tokens_of)
        seen.append(fb.split_seqs)
        return fb, sample

    monkeypatch.setattr(ModelRunner, "mixed_batch", counting)
    split, _, _, _ = _chunked_generate(0, 1, "llama-tiny", {}, False)
    assert any(s > 0 for s in seen), "the workload never mixed a continuation with fresh prompts"

    def unsplit(self, plan, tokens_of):
        fb, sample = orig(self, plan, tokens_of)
        fb.split_seqs = 0
        return fb, sample

    monkeypatch.setattr(ModelRunner, "mixed_batch", unsplit)
    whole, _, _, _ = _chunked_generate(0, 1, "llama-tiny", {}, False)
    assert split == whole
