"""ModelRunner: turns scheduler step plans into device batches and runs the stage, replaying
hipGraph-captured decode steps ("a single hipGraphLaunch per step per rank").

Decode graphs are captured per batch-size bucket on static input buffers; a step copies its
inputs into the bucket's buffers (padding rows: slot -1 = no cache write, ctx_len 1) and
replays. Everything inside — GEMMs, RoPE/KV append, paged attention, norms, TP all-reduces
(RCCL or the one-shot P2P kernel), the LM head and the TP sampling all-gather — is captured,
so the host cost per token is one replay.

Pipeline stages on native RCCL (`set_pipeline_io`): a non-first stage's decode graph starts
with the receive of the previous stage's boundary rows (Communicator.recv_native, captured in
the graph), landing them directly in the graph's static `hidden_in`; the full bucket is on the
wire, so sender and receiver agree on the shape whatever each replays. A stage that sends keeps
TWO instances per bucket and alternates them: the send of one instance's static output (issued
by the engine on the communicator's send stream, no copy) may still be in flight while the
other instance computes the next tick; an instance is replayed again only after its send-done
event (`_DecodeGraph.send_done`).
"""
from __future__ import annotations

import bisect
import os
from typing import Optional

import numpy as np
import torch

from .. import ops
from .batch import ForwardBatch


def _to_dev(a, dev) -> torch.Tensor:
    """Host array (staged through numpy) or a tensor already on the device (e.g. input ids
    gathered from the previous pipeline tick's broadcast) -> tensor on `dev`."""
    if isinstance(a, torch.Tensor):
        return a.to(dev, non_blocking=True)
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=True)


def _recover_from_capture(device) -> None:
    """After a failed capture: wait for the device and clear the sticky capture error, so the
    eager fallback's first launch does not report it as its own."""
    try:
        torch.cuda.synchronize(device)
    except Exception:  # noqa: BLE001 — the error being cleared may surface here first
        pass
    if ops.load_library():
        torch.ops.bfly.hip_clear_error()


class _DecodeGraph:
    """Static inputs / output of one decode graph (bucket). The inputs are views of ONE int32
    device buffer [ids | positions | slots | ctx_lens | block tables | temperatures (f32 bits)
    | seeds (int64)], so a step stages them with a single host-to-device copy from a pinned
    buffer (two, alternating, each reused only after the event of its previous copy). A last
    stage's graph ends with the sampling kernel (and the TP merge) on those per-request
    temperatures / seeds: `ids` are the step's tokens, one replay per step."""

    def __init__(self, bucket: int, max_blocks: int, device, hidden: int, first: bool):
        b = bucket
        self.bucket = bucket
        self.max_blocks = max_blocks
        self.off_t = b * (4 + max_blocks)                 # temperatures
        self.off_s = (self.off_t + b + 1) // 2 * 2        # seeds: 8-byte aligned int32 offset
        # initial state built on the host and copied once: padding rows have no cache slot (-1)
        # and context 1 (no torch fill kernels on the device)
        init = torch.zeros(self.off_s + 2 * b, dtype=torch.int32)
        init[2 * b:3 * b] = -1
        init[3 * b:4 * b] = 1
        self.inbuf = init.to(device)
        self.input_ids = self.inbuf[0:b]
        self.positions = self.inbuf[b:2 * b]
        self.slots = self.inbuf[2 * b:3 * b]
        self.ctx_lens = self.inbuf[3 * b:4 * b]
        self.block_tables = self.inbuf[4 * b:self.off_t].view(b, max_blocks)
        self.temps = self.inbuf[self.off_t:self.off_t + b].view(torch.float32)
        self.seeds = self.inbuf[self.off_s:self.off_s + 2 * b].view(torch.int64)
        self.ids: Optional[torch.Tensor] = None     # sampled in the graph (last stage)
        pin = torch.cuda.is_available() and torch.device(device).type == "cuda"
        self.host = [torch.zeros(self.inbuf.numel(), dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.host_np = [h.numpy() for h in self.host]
        self.host_events = [None, None]
        self.host_flip = 0
        self.hidden_in = None if first else torch.zeros(bucket, hidden, dtype=torch.bfloat16).to(device)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.output: Optional[torch.Tensor] = None
        self.send_done = None        # event: the send of `output` has completed (pipeline stages)


class ModelRunner:
    def __init__(self, model, kv_cache, max_seq_len: int, use_graphs: bool = True,
                 graph_batch_sizes: Optional[list] = None, post_fn=None, max_batch: int = 256):
        """`post_fn(output) -> tensor` is captured together with the forward when given (e.g.
        the TP sampler), so the replay returns the sampled ids directly."""
        self.model = model
        self.kv = kv_cache
        self.device = model.device
        self.max_seq_len = max_seq_len
        self.block_size = kv_cache.block_size
        self.max_blocks = (max_seq_len + self.block_size - 1) // self.block_size
        self.use_graphs = use_graphs and self.device.type == "cuda" and \
            os.environ.get("BFLY_DISABLE_GRAPHS", "0") != "1"
        self.buckets = sorted(graph_batch_sizes or [1, 2, 4, 8, 16, 32, 64])
        self.graphs: dict[int, _DecodeGraph] = {}
        self.eager_buckets: set = set()
        self.pool = None
        self.post_fn = post_fn
        # BFLY_PROGRAM_CHECK: rows -> the in-stage collectives of this rank's decode-step
        # program (engine._program_check); decode forwards run under comm.expect(...)
        self.conform = None
        # host staging buffers (pinned) for per-step inputs
        hb = max(self.buckets + [max_batch])
        self._tables_host = np.zeros((hb, self.max_blocks), dtype=np.int32)
        self._ctx_host = np.zeros((hb,), dtype=np.int32)
        # native pipeline I/O (set_pipeline_io)
        self.recv_fn = None
        self.instances = 1
        # sample_fn(logits, temps, seeds) -> ids, captured at the end of a last stage's decode
        # graphs (set by the engine); last_ids: the ids of the latest graph replay, else None
        self.sample_fn = None
        self.last_ids: Optional[torch.Tensor] = None
        self._flip: dict = {}          # bucket -> index of the instance replayed next
        self.last_instance: Optional[_DecodeGraph] = None

    def set_pipeline_io(self, recv_fn=None, sends: bool = False) -> None:
        """`recv_fn(t)`: receive the previous stage's rows into `t` on the current stream
        (captured at the head of every decode graph); `sends`: the stage's outputs are sent,
        so each bucket gets two alternating instances (module doc)."""
        self.recv_fn = recv_fn
        self.instances = 2 if sends else 1

    def bucket_of(self, n: int) -> int:
        return self.buckets[bisect.bisect_left(self.buckets, n)]

    # ------------------------------------------------------------------------------------
    def prefill_batch(self, plan, tokens_of) -> ForwardBatch:
        """Batch for a prefill plan; tokens_of(sid) -> full token list to (re)compute."""
        ids, pos, slots, cu, last = [], [], [], [0], []
        for sid, sl in zip(plan.seq_ids, plan.prefill_slots):
            toks = tokens_of(sid)
            n = len(sl)
            ids.extend(toks[:n])
            pos.extend(range(n))
            slots.extend(sl)
            cu.append(cu[-1] + n)
            last.append(cu[-1] - 1)
        dev = self.device
        i32 = dict(dtype=torch.int32)
        return ForwardBatch(
            input_ids=torch.tensor(ids, **i32).to(dev, non_blocking=True),
            positions=torch.tensor(pos, **i32).to(dev, non_blocking=True),
            slots=torch.tensor(slots, **i32).to(dev, non_blocking=True), is_prefill=True,
            cu_seqlens=torch.tensor(cu, **i32).to(dev, non_blocking=True),
            max_seqlen=max(cu[i + 1] - cu[i] for i in range(len(cu) - 1)),
            logits_idx=torch.tensor(last, dtype=torch.int64).to(dev, non_blocking=True))

    def mixed_batch(self, plan, tokens_of) -> tuple:
        """Batch of a mixed / chunked-prefill step (runtime/scheduler.cpp mixed mode): decode
        rows first, then each scheduled prompt chunk. Returns (batch, rids whose row is
        sampled: every decode row and the last row of every chunk that completes its prompt)."""
        nd = plan.num_decode
        sids = list(plan.seq_ids)
        dec = sids[:nd]
        ids = [tokens_of(s)[-1] for s in dec]
        pos = list(plan.decode_positions)
        slots = list(plan.decode_slots)
        rows, sample = list(range(nd)), list(dec)
        cu, prefix, chunk_sids = [0], [], sids[nd:]
        for j, sid in enumerate(chunk_sids):
            st, n = int(plan.prefill_starts[j]), int(plan.prefill_lens[j])
            ids.extend(tokens_of(sid)[st:st + n])
            pos.extend(range(st, st + n))
            slots.extend(plan.prefill_slots[j])
            cu.append(cu[-1] + n)
            prefix.append(st)
            if plan.prefill_final[j]:
                rows.append(nd + cu[-1] - 1)
                sample.append(sid)
        dev = self.device
        t32 = lambda a: torch.tensor(a, dtype=torch.int32).to(dev, non_blocking=True)  # noqa: E731
        bt = ctx = pre_cu = pre_tab = None
        if nd:
            self.kv.manager.fill_decode_tables(dec, self._tables_host[:nd], self._ctx_host[:nd])
            bt = torch.from_numpy(self._tables_host[:nd].copy()).to(dev, non_blocking=True)
            ctx = torch.from_numpy(self._ctx_host[:nd].copy()).to(dev, non_blocking=True)
        if any(prefix):
            pc = [0]
            for p in prefix:
                pc.append(pc[-1] + p)
            pre_cu = t32(pc)
            # every chunk's full table (prefix pages and the chunk's own): the paged prefill
            # attention reads the chunk's keys from the cache too
            tab = np.zeros((len(chunk_sids), self.max_blocks), dtype=np.int32)
            for j, sid in enumerate(chunk_sids):
                b = self.kv.manager.block_table(sid)
                tab[j, : len(b)] = b
            pre_tab = torch.from_numpy(tab).to(dev, non_blocking=True)
        lens = [cu[i + 1] - cu[i] for i in range(len(cu) - 1)]
        fb = ForwardBatch(input_ids=t32(ids), positions=t32(pos), slots=t32(slots), is_prefill=True,
                          cu_seqlens=t32(cu), max_seqlen=max(lens, default=0),
                          block_tables=bt, ctx_lens=ctx, max_ctx=self.max_seq_len,
                          logits_idx=torch.tensor(rows, dtype=torch.int64).to(dev, non_blocking=True),
                          num_decode=nd, prefix_lens=prefix if any(prefix) else None, prefix_cu=pre_cu,
                          prefix_tables=pre_tab)
        # continuation chunks first, fresh prompts after them (the scheduler's order when it
        # resumes a partly prefilled prompt): only the continuations need the paged pass
        s1 = next((j for j, p in enumerate(prefix) if p == 0), len(prefix))
        if 0 < s1 < len(prefix) and not any(prefix[s1:]):
            fb.split_seqs, fb.split_rows = s1, cu[s1]
            fb.cu_fresh = t32([c - cu[s1] for c in cu[s1:]])
            fb.max_paged, fb.max_fresh = max(lens[:s1]), max(lens[s1:])
        return fb, sample

    def decode_inputs(self, plan, last_tokens: list) -> dict:
        B = len(plan.seq_ids)
        self.kv.manager.fill_decode_tables(list(plan.seq_ids), self._tables_host[:B], self._ctx_host[:B])
        ids = last_tokens if isinstance(last_tokens, torch.Tensor) else np.asarray(last_tokens, dtype=np.int32)
        return dict(ids=ids,
                    pos=np.asarray(plan.decode_positions, dtype=np.int32),
                    slots=np.asarray(plan.decode_slots, dtype=np.int32),
                    tables=self._tables_host[:B], ctx=self._ctx_host[:B])

    def decode_batch(self, inp: dict, ep_tokens: int = 0) -> ForwardBatch:
        dev = self.device
        t = lambda a: _to_dev(a, dev)  # noqa: E731
        return ForwardBatch(input_ids=t(inp["ids"]), positions=t(inp["pos"]), slots=t(inp["slots"]),
                            is_prefill=False, block_tables=t(inp["tables"]), ctx_lens=t(inp["ctx"]),
                            max_ctx=self.max_seq_len, logits_idx=None, ep_tokens=ep_tokens)

    # ------------------------------------------------------------------------------------
    def run(self, fb: ForwardBatch, hidden_in=None):
        if self.conform is not None and not fb.is_prefill and not getattr(fb, "ep_alltoall", False):
            # decode programs only: a decode step beside an EP peer's prefill (ep_alltoall) runs
            # the prefill exchange instead. EP ranks pad their exchange to the agreed row count
            # (fb.ep_tokens), which is the program's row count
            with self.model.comm.expect(self.conform(max(fb.num_tokens, fb.ep_tokens or 0))):
                out = self.model.forward(fb, self.kv.layers, hidden_in)
        else:
            out = self.model.forward(fb, self.kv.layers, hidden_in)
        return self.post_fn(out) if (self.post_fn is not None and self.model.last) else out

    def run_decode(self, inp: dict, hidden_in=None, ep_tokens: int = 0, graphs_ok: bool = True,
                   ep_alltoall: bool = False):
        """Decode step. With expert parallelism every EP rank must pad to the same row count
        (`ep_tokens`): the graph bucket is chosen from it, so all EP ranks replay the same
        shape; steps where some EP rank is prefilling run eagerly (graphs_ok=False)."""
        B = len(inp["ids"])
        need = max(B, ep_tokens)
        self.last_ids = None
        if self.recv_fn is not None or self.instances > 1:
            if need > self.buckets[-1]:
                raise RuntimeError(f"pipeline decode of {need} rows exceeds the largest bucket {self.buckets[-1]}")
            return self._run_pipeline_decode(self.bucket_of(need), inp, hidden_in)
        if not self.use_graphs or not graphs_ok or need > self.buckets[-1] or ep_alltoall:
            fb = self.decode_batch(inp, ep_tokens)
            fb.ep_alltoall = ep_alltoall
            return self.run(fb, hidden_in)
        bucket = self.buckets[bisect.bisect_left(self.buckets, need)]
        if bucket in self.eager_buckets:
            return self.run(self.decode_batch(inp, ep_tokens), hidden_in)
        g = self.graphs.get(bucket)
        if g is None:
            try:
                g = self._capture(bucket)
            except Exception as e:  # capture unsupported here (e.g. a collective): stay eager
                import warnings

                warnings.warn(f"hipGraph capture of decode bucket {bucket} failed ({e!r}); running eagerly")
                self.eager_buckets.add(bucket)
                _recover_from_capture(self.device)
                return self.run(self.decode_batch(inp, ep_tokens), hidden_in)
        self._stage(g, inp, hidden_in)
        g.graph.replay()
        if g.ids is not None:
            self.last_ids = g.ids[:B]
        return g.output[:B]

    def precapture(self, rows: int) -> bool:
        """Capture the decode graph of the bucket `rows` rows use now rather than inside the
        first decode step (as a server does at start-up). Single-stage runners only: a pipeline
        stage's graphs hold their receives. The capture's warm-up runs issue the step's
        collectives, so every rank of a TP / EP group must call it together."""
        if self.recv_fn is not None or self.instances > 1 or not self.use_graphs or rows > self.buckets[-1]:
            return False
        bucket = self.buckets[bisect.bisect_left(self.buckets, rows)]
        if bucket in self.graphs or bucket in self.eager_buckets:
            return bucket in self.graphs
        try:
            self._capture(bucket)
        except Exception as e:  # noqa: BLE001 — the first decode step then runs eagerly too
            import warnings

            warnings.warn(f"hipGraph capture of decode bucket {bucket} failed ({e!r}); running eagerly")
            self.eager_buckets.add(bucket)
            _recover_from_capture(self.device)
            return False
        return True

    def _run_pipeline_decode(self, bucket: int, inp: dict, hidden_in):
        """Decode of a pipeline stage with native I/O: alternate the bucket's instances, wait
        for the instance's previous send, receive (inside the graph, or eagerly into the same
        static buffer on the eager fallback) and run over the whole bucket. The instance is
        left in `last_instance` (its full-bucket `output` is what the engine sends)."""
        B = len(inp["ids"])
        insts = self.graphs.get(bucket)
        if insts is None:
            insts = []
            for i in range(self.instances):
                g = None
                if self.use_graphs and bucket not in self.eager_buckets:
                    try:
                        g = self._capture(bucket, register=False)
                    except Exception as e:  # noqa: BLE001 — eager on the same static buffers
                        import warnings

                        warnings.warn(f"hipGraph capture of decode bucket {bucket} failed ({e!r}); "
                                      "running eagerly")
                        self.eager_buckets.add(bucket)
                        _recover_from_capture(self.device)
                if g is None:
                    m = self.model
                    g = _DecodeGraph(bucket, self.max_blocks, self.device, m.cfg.hidden_size, m.first)
                insts.append(g)
            self.graphs[bucket] = insts
        i = self._flip.get(bucket, 0)
        self._flip[bucket] = (i + 1) % len(insts)
        g = insts[i]
        if g.send_done is not None:
            torch.cuda.current_stream(self.device).wait_event(g.send_done)
            g.send_done = None
        self._stage(g, inp, None if self.recv_fn is not None else hidden_in)
        if g.graph is not None:
            g.graph.replay()
            if g.ids is not None:
                self.last_ids = g.ids[:B]
        else:
            if self.recv_fn is not None:
                self.recv_fn(g.hidden_in)
            g.output = self.run(self._graph_batch(g), g.hidden_in)
        self.last_instance = g
        return g.output[:B]

    def _stage(self, g: _DecodeGraph, inp: dict, hidden_in) -> None:
        """Fill the graph's static inputs: the host arrays (padding rows included: position 0,
        no cache slot, context 1, page 0) go into a pinned buffer and reach the device in one
        copy; input ids already on the device (gathered from the previous step's sampled ids)
        are copied device to device."""
        B, b = len(inp["ids"]), g.bucket
        k = g.host_flip
        g.host_flip ^= 1
        if g.host_events[k] is not None:
            g.host_events[k].synchronize()        # its previous copy has read the buffer
        h = g.host_np[k]
        ids = inp["ids"]
        ids_dev = isinstance(ids, torch.Tensor) and ids.device.type != "cpu"
        if not ids_dev:
            h[0:B] = ids.numpy() if isinstance(ids, torch.Tensor) else ids
            h[B:b] = 0
        h[b:b + B] = inp["pos"]
        h[b + B:2 * b] = 0
        h[2 * b:2 * b + B] = inp["slots"]
        h[2 * b + B:3 * b] = -1
        h[3 * b:3 * b + B] = inp["ctx"]
        h[3 * b + B:4 * b] = 1
        tab = h[4 * b:g.off_t].reshape(b, g.max_blocks)
        tab[:B] = inp["tables"]
        tab[B:] = 0
        ht = h[g.off_t:g.off_t + b].view(np.float32)
        hs = h[g.off_s:g.off_s + 2 * b].view(np.int64)
        t, sd = inp.get("temps"), inp.get("seeds")
        ht[:B] = 0.0 if t is None else t
        ht[B:] = 0.0
        hs[:B] = 0 if sd is None else sd
        hs[B:] = 0
        start = b if ids_dev else 0
        g.inbuf[start:].copy_(g.host[k][start:], non_blocking=True)
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            g.host_events[k] = ev
        if ids_dev:
            g.input_ids[:B].copy_(ids)
            if B < b:
                ops.zero_(g.input_ids[B:])
        if g.hidden_in is not None and hidden_in is not None:
            g.hidden_in[:B].copy_(hidden_in)

    def _graph_batch(self, g: _DecodeGraph) -> ForwardBatch:
        return ForwardBatch(input_ids=g.input_ids, positions=g.positions, slots=g.slots,
                            is_prefill=False, block_tables=g.block_tables, ctx_lens=g.ctx_lens,
                            max_ctx=self.max_seq_len, logits_idx=None, ep_tokens=g.bucket)

    def _capture(self, bucket: int, register: bool = True) -> _DecodeGraph:
        m = self.model
        g = _DecodeGraph(bucket, self.max_blocks, self.device, m.cfg.hidden_size, m.first)
        fb = self._graph_batch(g)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        sample = self.sample_fn if (self.sample_fn is not None and self.model.last) else None
        with torch.cuda.stream(s):
            for _ in range(2):   # warm up allocator / workspaces outside capture (no receive:
                out = self.run(fb, g.hidden_in)   # a transfer would consume a real message)
                if sample is not None:
                    sample(out, g.temps, g.seeds)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self.pool):
            if self.recv_fn is not None and g.hidden_in is not None:
                self.recv_fn(g.hidden_in)       # the boundary receive is the graph's first node
            g.output = self.run(fb, g.hidden_in)
            if sample is not None:
                g.ids = sample(g.output, g.temps, g.seeds)
        g.graph = graph
        if register:
            self.graphs[bucket] = g
        return g

    def close(self) -> None:
        """Drop every captured graph and the graph memory pool (before the communicators whose
        kernels the graphs captured are torn down: parallel/rccl.py)."""
        for v in self.graphs.values():
            for g in (v if isinstance(v, list) else [v]):
                g.graph = None
                g.send_done = None
        self.graphs.clear()
        self.last_instance = None
        self.pool = None
        import gc

        gc.collect()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def capture_all(self, max_batch: int) -> None:
        for b in self.buckets:
            if b <= max_batch and b not in self.graphs:
                self._capture(b)

    @property
    def captured_buckets(self) -> list:
        return sorted(b for b, g in self.graphs.items()
                      if (g.graph is not None if isinstance(g, _DecodeGraph) else all(x.graph is not None for x in g)))
