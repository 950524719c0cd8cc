"""Pipeline boundary on native RCCL inside the stage graph, on one MI355X:

* a ONE-rank native communicator sends to and receives from itself inside group_start/end,
  captured in a hipGraph and replayed with new payloads, against the eager transfer;
* ModelRunner.set_pipeline_io: a non-first stage's decode graph starts with the receive (here
  a captured stand-in copy from a static source), lands the rows in its static hidden_in, and
  a sending stage alternates two instances guarded by send-done events; every replay equals
  the eager stage forward over the same bucket-padded rows.
(RCCL refuses two ranks on one device: the two-rank edge runs on the driver's 8-GPU node, after
the preflight's pp_edge_graph check has run exactly this pattern across the ranks.)"""
import time

import pytest
import torch

from butterfly_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _lib():
    assert ops.load_library(), ops._load_error


def test_self_send_recv_captured_in_graph():
    from butterfly_amd.parallel.rccl import RcclComm

    c = RcclComm.create(torch.ops.bfly.rccl_unique_id(), 1, 0)
    try:
        src = torch.zeros(64, 8192, dtype=torch.bfloat16, device="cuda")
        dst = torch.zeros_like(src)

        def xfer():
            RcclComm.group_start()
            c.send(src, 0)
            c.recv(dst, 0)
            RcclComm.group_end()

        src.normal_()
        xfer()                                  # eager
        torch.cuda.synchronize()
        assert torch.equal(dst, src)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            xfer()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            src.mul_(2.0)                       # producer kernel -> transfer -> consumer kernel
            xfer()
            dst.add_(1.0)
        for _ in range(3):
            src.normal_()
            want = src.float() * 2 + 1
            g.replay()
            torch.cuda.synchronize()
            torch.testing.assert_close(dst.float(), want.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
        assert c.async_error() == 0
        # teardown in the engine's order: the graph that captured the transfer first, then a
        # bounded finalize + destroy of the communicator (non-blocking: it cannot hang)
        del g
        torch.cuda.synchronize()
        t0 = time.monotonic()
        status = c.close(timeout=20.0)
        assert status == "clean", status
        assert time.monotonic() - t0 < 20.0
    finally:
        c.close(abort=True)          # no-op after the clean close


def _stage_model(first: bool):
    from butterfly_amd.config import ModelConfig
    from butterfly_amd.models import Shard, build_model

    cfg = ModelConfig.from_preset("llama-small")
    half = cfg.num_layers // 2
    shard = Shard(layer_start=0 if first else half, layer_end=half if first else cfg.num_layers)
    m = build_model(cfg, shard, device="cuda", dtype=torch.bfloat16)
    m.init_random(seed=5)
    return cfg, m


@pytest.mark.parametrize("graphs", [True, False])
def test_runner_receives_in_graph_and_alternates_instances(graphs):
    from butterfly_amd.engine.kv_cache import KVCache
    from butterfly_amd.engine.model_runner import ModelRunner

    cfg, m = _stage_model(first=False)
    bs = 32
    kv = KVCache(m, 64, bs, torch.bfloat16)
    runner = ModelRunner(m, kv, 256, use_graphs=graphs, graph_batch_sizes=[4, 8], max_batch=8)
    wire = torch.zeros(8, cfg.hidden_size, dtype=torch.bfloat16, device="cuda")   # the "previous stage"
    runner.set_pipeline_io(recv_fn=lambda t: t.copy_(wire[: t.shape[0]]), sends=True)
    B = 3
    import numpy as np

    tables = np.zeros((B, runner.max_blocks), dtype=np.int32)
    for i in range(B):
        tables[i, :2] = [2 * i, 2 * i + 1]
    inp = dict(ids=np.zeros(B, dtype=np.int32), pos=np.array([5, 9, 17], dtype=np.int32),
               slots=np.array([2 * i * bs + p for i, p in enumerate([5, 9, 17])], dtype=np.int32),
               tables=tables, ctx=np.array([6, 10, 18], dtype=np.int32))
    seen = []
    for step in range(4):
        wire.normal_()
        out = runner.run_decode(inp, None)
        g = runner.last_instance
        assert out.shape[0] == B and g.output.shape[0] == 4          # bucket rows on the wire
        seen.append(id(g))
        ev = torch.cuda.Event()
        ev.record()
        g.send_done = ev                                           # as the engine's send would
        # eager reference over the same bucket-padded rows
        ref = runner.run(runner._graph_batch(g), wire[:4].clone())
        torch.cuda.synchronize()
        torch.testing.assert_close(g.output.float(), ref.float(), rtol=2e-2, atol=2e-2)
    assert seen[0] == seen[2] and seen[1] == seen[3] and seen[0] != seen[1]   # A/B alternation
    if graphs:
        assert runner.captured_buckets == [4]
