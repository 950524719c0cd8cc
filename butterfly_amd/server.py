"""HTTP serving front end (OpenAI-style /v1/completions), rank 0 only.

Serving is SPMD like everything else: every rank of the job runs a `ServingLoop`. Rank 0 also
runs the HTTP server; its handlers enqueue requests. At the top of every engine step rank 0
broadcasts the newly arrived requests (and a shutdown flag) to all ranks over a gloo control
group, every rank adds them to its engine in the same order, and all ranks take the step
together — identical scheduler inputs on every rank, so identical step plans (the engine's
determinism contract, engine/engine.py). Data-parallel replicas: rank 0 assigns each request
to a replica round-robin; replicas that get nothing simply step idle.

Streaming (`"stream": true`, OpenAI server-sent events): the stream flag travels with the
request broadcast, so each replica's leader also reports the tokens its streaming requests
gained in the step; rank 0 pushes them into the request's queue and the HTTP handler emits one
`data:` event per token, then a final event with the finish reason and `data: [DONE]`.
"""
from __future__ import annotations

import asyncio
import itertools
import queue
import threading
import time
from typing import Optional

import torch.distributed as dist

from .engine.sampler import SamplingParams
from .utils.logging import get_logger

log = get_logger("server")


class ServingLoop:
    def __init__(self, llm, idle_sleep: float = 0.002):
        self.llm = llm
        self.engine = llm.engine
        self.rank = llm.rank
        self.world = llm.world
        self.inbox: "queue.Queue" = queue.Queue()
        self.waiters: dict = {}
        self.results: dict = {}
        self.streams: dict = {}          # rank 0: gid -> queue of ("token", id) / ("done", result)
        self.streaming: set = set()      # every rank: gids whose tokens are reported per step
        self.idle_sleep = idle_sleep
        self.stop = False
        self._ids = itertools.count()
        self._dp_rr = itertools.count()
        self.ctrl = dist.new_group(backend="gloo") if self.world > 1 else None

    # rank 0: called from HTTP handlers (any thread)
    def submit(self, token_ids: list, params: SamplingParams, stream: bool = False) -> int:
        gid = next(self._ids)
        ev = threading.Event()
        self.waiters[gid] = ev
        if stream:
            self.streams[gid] = queue.Queue()
        self.inbox.put((gid, list(token_ids), params, next(self._dp_rr) % self.llm.plan.dp, stream))
        return gid

    def stream_events(self, gid: int, timeout: float = 600.0):
        """Blocking iterator over ("token", id) ... ("done", result) for a streaming request."""
        q = self.streams[gid]
        try:
            while True:
                kind, val = q.get(timeout=timeout)
                yield kind, val
                if kind == "done":
                    return
        finally:
            self.streams.pop(gid, None)
            self.waiters.pop(gid, None)
            self.results.pop(gid, None)

    def wait(self, gid: int, timeout: Optional[float] = None) -> dict:
        self.waiters[gid].wait(timeout)
        self.waiters.pop(gid, None)
        return self.results.pop(gid)

    def _exchange(self) -> tuple:
        new = []
        if self.rank == 0:
            while True:
                try:
                    new.append(self.inbox.get_nowait())
                except queue.Empty:
                    break
        if self.world > 1:
            obj = [(new, self.stop)]
            dist.broadcast_object_list(obj, src=0, group=self.ctrl)
            new, stop = obj[0]
        else:
            stop = self.stop
        return new, stop

    def run(self) -> None:
        eng = self.engine
        my_dp = self.llm.dp_rank
        c = self.llm.plan.mesh.coord(self.rank)
        leader = c.tp == 0 and c.pp == 0          # one reporter per data-parallel replica
        while True:
            new, stop = self._exchange()
            for gid, ids, params, dp, stream in new:
                if dp == my_dp:
                    eng.add_request(ids, params, rid=gid)
                    if stream:
                        self.streaming.add(gid)
            if stop and self._all_idle():      # collective: every rank evaluates it
                return
            finished, tokens = [], []
            if eng.has_unfinished() or eng.lockstep_dp:
                out = eng.step()
                if self.streaming:
                    tokens = [(r, t) for r, t in zip(out.rids, out.new_tokens) if r in self.streaming]
                for rid in out.finished:
                    self.streaming.discard(rid)
                    req = eng.requests.pop(rid)
                    finished.append((rid, {"token_ids": list(req.output), "finish_reason": req.finish_reason,
                                           "ttft_s": req.first_token_time - req.arrival if req.first_token_time else None,
                                           "e2e_s": req.finish_time - req.arrival}))
            elif not new:
                time.sleep(self.idle_sleep)
            if self.world > 1:
                got = [None] * self.world if self.rank == 0 else None
                dist.gather_object((finished, tokens) if leader else ([], []), got, dst=0, group=self.ctrl)
                if self.rank == 0:
                    finished = [x for f, _ in got for x in f]
                    tokens = [x for _, t in got for x in t]
            if self.rank == 0:
                for rid, tok in tokens:
                    q = self.streams.get(rid)
                    if q is not None:
                        q.put(("token", int(tok)))
                for rid, res in finished:
                    self._publish(rid, res)

    def _all_idle(self) -> bool:
        if self.world == 1:
            return True
        t = [int(self.engine.has_unfinished())]
        out = [None] * self.world
        dist.all_gather_object(out, t, group=self.ctrl)
        return not any(o[0] for o in out)

    def _publish(self, rid, res) -> None:
        q = self.streams.get(rid)
        if q is not None:
            q.put(("done", res))
            return
        self.results[rid] = res
        ev = self.waiters.get(rid)
        if ev:
            ev.set()


def _request_model(BaseModel):
    # built at runtime (pydantic is imported lazily); annotations are real types, not strings
    ns = {"__annotations__": {"model": Optional[str], "prompt": object, "max_tokens": int, "temperature": float,
                              "top_p": float, "top_k": int, "seed": Optional[int], "stop_token_ids": list,
                              "stream": bool},
          "model": None, "max_tokens": 16, "temperature": 0.0, "top_p": 1.0, "top_k": 0, "seed": None,
          "stop_token_ids": [], "stream": False}
    return type("CompletionRequest", (BaseModel,), ns)


def create_app(loop: ServingLoop):
    import json

    from fastapi import FastAPI, HTTPException
    from fastapi.responses import PlainTextResponse, StreamingResponse
    from pydantic import BaseModel

    app = FastAPI(title="butterfly_amd")
    tok = loop.llm.tokenizer

    CompletionRequest = _request_model(BaseModel)

    @app.get("/health")
    def health():
        return {"status": "ok", "rank": loop.rank, "world": loop.world, "plan": loop.llm.plan.name}

    @app.get("/v1/models")
    def models():
        return {"object": "list", "data": [{"id": loop.llm.cfg.name, "object": "model"}]}

    @app.get("/metrics", response_class=PlainTextResponse)
    def metrics():
        return loop.engine.metrics.to_prometheus()

    async def completions(req):
        if isinstance(req.prompt, str):
            ids, is_text = tok.encode(req.prompt), True
        elif isinstance(req.prompt, list) and all(isinstance(i, int) for i in req.prompt):
            ids, is_text = req.prompt, False
        else:
            raise HTTPException(400, "prompt must be a string or a list of token ids")
        params = SamplingParams(max_tokens=req.max_tokens, temperature=req.temperature, top_p=req.top_p,
                                top_k=req.top_k, seed=req.seed, stop_token_ids=req.stop_token_ids)
        if req.stream:
            gid = loop.submit(ids, params, stream=True)

            def sse():   # runs in Starlette's threadpool: the blocking queue reads are fine
                for kind, val in loop.stream_events(gid):
                    if kind == "token":
                        chunk = {"index": 0, "token_ids": [val], "text": tok.decode([val]) if is_text else None,
                                 "finish_reason": None}
                    else:
                        chunk = {"index": 0, "token_ids": [], "text": "" if is_text else None,
                                 "finish_reason": val["finish_reason"]}
                    ev = {"id": f"cmpl-{gid}", "object": "text_completion", "model": loop.llm.cfg.name,
                          "choices": [chunk]}
                    yield f"data: {json.dumps(ev)}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(sse(), media_type="text/event-stream")
        gid = loop.submit(ids, params)
        res = await asyncio.get_running_loop().run_in_executor(None, loop.wait, gid, 600.0)
        text = tok.decode(res["token_ids"]) if is_text else None
        return {"id": f"cmpl-{gid}", "object": "text_completion", "model": loop.llm.cfg.name,
                "choices": [{"index": 0, "text": text, "token_ids": res["token_ids"],
                             "finish_reason": res["finish_reason"]}],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(res["token_ids"])},
                "timing": {"ttft_s": res["ttft_s"], "e2e_s": res["e2e_s"]}}

    completions.__annotations__ = {"req": CompletionRequest}
    app.post("/v1/completions")(completions)
    return app


def serve(llm, host: str = "127.0.0.1", port: int = 8000) -> None:
    loop = ServingLoop(llm)
    if llm.rank != 0:
        loop.run()
        return
    import uvicorn

    th = threading.Thread(target=loop.run, name="bfly-engine", daemon=True)
    th.start()
    try:
        uvicorn.run(create_app(loop), host=host, port=port, log_level="warning")
    finally:
        loop.stop = True
        th.join(timeout=30)
