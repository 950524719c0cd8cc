"""Process launcher: one process per GPU (SURVEY.md §3.2 (1) `bfly launch -n 8 -- ...`).

Starts `nproc` child processes with the torch.distributed environment (RANK, WORLD_SIZE,
LOCAL_RANK, MASTER_ADDR=127.0.0.1, MASTER_PORT, HSA_ENABLE_IPC_MODE_LEGACY=0 for dmabuf IPC),
prefixes each child's output with its rank, and fails fast: when any rank exits non-zero the
others are terminated and the launcher returns that code (or, with --max-restarts, starts the
whole job again: restart-based recovery on top of request-state snapshots). The launcher itself
never touches the GPU, so it can start GPU programs safely.

`placement` (a PartitionPlan's mesh rank -> GPU index map, `launch --plan plan.json`) sets each
rank's LOCAL_RANK, the device index every entry point binds (init_distributed -> set_device and
the RCCL communicator's device). The partitioner emits the identity on the fully connected
xGMI mesh (partition/search.py), but a hand-edited plan is honoured.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(stream, prefix: str, out) -> None:
    for line in iter(stream.readline, b""):
        out.write(prefix + line.decode(errors="replace"))
        out.flush()


def launch(cmd: list, nproc: int, master_port: int | None = None, env_extra: dict | None = None,
           prefix_output: bool = True, placement: list | None = None, max_restarts: int = 0) -> int:
    """Run the job; with `max_restarts` > 0 a failed job (any rank non-zero, the rest taken
    down) is started again, whole, up to that many times, with BFLY_RESTART=<attempt> in its
    environment. Programs that snapshot their request state (EngineConfig.snapshot_every,
    engine/state.py) resume from it on a restart (`generate --snapshot-dir`), so a rank failure
    costs the steps since the last snapshot, not the requests."""
    if placement is not None and sorted(placement) != list(range(nproc)):
        raise ValueError(f"placement {placement} is not a permutation of 0..{nproc - 1}")
    code = 0
    for attempt in range(max_restarts + 1):
        if attempt:
            print(f"[launch] job failed with exit code {code}; restart {attempt}/{max_restarts}",
                  file=sys.stderr, flush=True)
        extra = dict(env_extra or {}, BFLY_RESTART=str(attempt))
        # a fixed port only for the first attempt: the old job's sockets may linger
        code = _run_once(cmd, nproc, master_port if attempt == 0 else None, extra, prefix_output, placement)
        if code == 0 or code == 130:
            break
    return code


def _run_once(cmd: list, nproc: int, master_port: int | None, env_extra: dict, prefix_output: bool,
              placement: list | None) -> int:
    port = master_port or _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        dev = placement[r] if placement is not None else r
        env.update(RANK=str(r), LOCAL_RANK=str(dev), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.update(env_extra)
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if prefix_output else None,
                             stderr=subprocess.STDOUT if prefix_output else None, start_new_session=True)
        procs.append(p)
        if prefix_output:
            threading.Thread(target=_pump, args=(p.stdout, f"[rank{r}] ", sys.stdout), daemon=True).start()
    code = 0
    try:
        while procs:
            for p in list(procs):
                rc = p.poll()
                if rc is None:
                    continue
                procs.remove(p)
                if rc != 0 and code == 0:
                    code = rc
                    for q in procs:          # fail fast: take the rest of the job down
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            os.killpg(q.pid, signal.SIGTERM)
        code = 130
    return code
