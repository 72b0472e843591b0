"""Rank supervisor for multi-process runs: a multi-GPU run that cannot end without a number or a reason.

`bench.py --gpus N` runs one process per GPU (torch.distributed.run, or bench.py's own launcher). Each of those rank
processes is a supervisor: it never touches the GPU (no HIP call, no torch.cuda), and runs the real rank as a child
process, attempt by attempt:

  attempt 0: the combines over RCCL (device all-gathers, after the bit-exact self-check of shyft_amd.distributed);
  attempt 1: the same run with every combine over gloo (host copies of the [C][T] partials).

A child that exits non-zero, or makes no progress for a while (the worker prints progress markers on stderr: rendezvous,
self-check, every chunk), ends its attempt: the supervisors agree over a TCP store (torchrun's agent store, or one rank 0
hosts) and start the next attempt with fresh children on a fresh rendezvous port -- a process that touched the GPU is
never re-executed, it is killed and replaced by a new child. Rank 0's JSON line is forwarded as soon as its child prints
it; once it has been printed the run is done, whatever the teardown does. The line of a fallback attempt says which
attempt produced it and why the previous one ended (`supervisor` field).

The reference runs the whole region in one process (core/region_model.h:991-1021), so it has no exchange to stall on;
this is the guard the multi-process split needs.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time

PROGRESS_TAG = "[shyft-progress]"
ATTEMPTS = (("rccl", {}), ("gloo", {"SHYFT_DIST_BACKEND": "gloo"}))


def progress(name: str) -> None:
    """Worker side: one liveness marker for the supervisor (no-op when not supervised)."""
    if os.environ.get("SHYFT_SUPERVISED") == "1":
        print(f"{PROGRESS_TAG} {name}", file=sys.stderr, flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _store(world: int, rank: int, timeout_s: float):
    from datetime import timedelta
    from torch.distributed import TCPStore
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ["MASTER_PORT"])
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"   # torchrun's agent hosts it
    return TCPStore(host, port, world, is_master=(rank == 0 and not agent), timeout=timedelta(seconds=timeout_s),
                    wait_for_workers=False)


class _Child:
    """One attempt's worker process: stdout forwarded line by line (rank 0's JSON line noticed), stderr forwarded and
    scanned for progress markers."""

    def __init__(self, argv, env):
        self.p = subprocess.Popen(argv, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, bufsize=1,
                                  start_new_session=True)
        self.last = time.monotonic()
        self.marks = 0
        self.line = False
        self.tail = []
        self._t = [threading.Thread(target=self._out, daemon=True), threading.Thread(target=self._err, daemon=True)]
        for t in self._t:
            t.start()

    def _out(self):
        for ln in self.p.stdout:
            sys.stdout.write(ln)
            sys.stdout.flush()
            self.last = time.monotonic()
            if ln.lstrip().startswith("{"):
                self.line = True

    def _err(self):
        for ln in self.p.stderr:
            if ln.startswith(PROGRESS_TAG):
                self.last = time.monotonic()
                self.marks += 1
                continue
            sys.stderr.write(ln)
            sys.stderr.flush()
            self.tail = (self.tail + [ln.rstrip()])[-5:]

    def poll(self):
        return self.p.poll()

    def kill(self):
        if self.p.poll() is None:
            try:
                os.killpg(self.p.pid, signal.SIGKILL)   # the child's own session: it and anything it started
            except ProcessLookupError:
                pass
        self.p.wait()
        for t in self._t:
            t.join(timeout=5)


def supervise(argv, attempts=ATTEMPTS) -> int:
    """Run `argv` (a worker command) as this rank's child, attempt by attempt; returns the exit status of the rank."""
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    first_s = float(os.environ.get("SHYFT_SUPERVISE_FIRST_S", "420"))   # first marker (a fresh box's first import)
    stall_s = float(os.environ.get("SHYFT_SUPERVISE_STALL_S", "240"))   # between markers
    store = _store(world, rank, timeout_s=first_s + stall_s + 600)
    reason = ""
    for a, (name, extra) in enumerate(attempts):
        key = f"shyft_supervise/{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}/{a}"
        if rank == 0:
            store.set(f"{key}/port", str(_free_port()))
        port = store.get(f"{key}/port").decode()
        env = dict(os.environ, MASTER_PORT=port, MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   TORCHELASTIC_USE_AGENT_STORE="False", SHYFT_SUPERVISED="1", SHYFT_SUPERVISE_ATTEMPT=str(a),
                   SHYFT_SUPERVISE_MODE=name, SHYFT_SUPERVISE_REASON=reason, **extra)
        child = _Child(argv, env)
        why = None
        decision = None
        while True:
            code = child.poll()
            now = time.monotonic()
            if store.check([f"{key}/decision"]):
                decision = store.get(f"{key}/decision").decode()
                break
            if rank == 0 and child.line:
                decision = "done"
                store.set(f"{key}/decision", decision)
                break
            if why is None:
                if code is not None and code != 0:
                    why = f"rank {rank} exited with status {code}" + (f" ({child.tail[-1][:200]})" if child.tail else "")
                elif code is None and now - child.last > (stall_s if child.marks else first_s):
                    why = f"rank {rank} made no progress for {int(now - child.last)} s"
                    child.kill()
                if why is not None:
                    store.set(f"{key}/fail/{rank}", why)
            if rank == 0 and (why is not None or code is not None):
                # rank 0 decides once its own child has ended without a line
                decision = ("retry" if a + 1 < len(attempts) else "fail") + ":" + (why or "no line printed")
                store.set(f"{key}/decision", decision)
                break
            if rank == 0 and why is None:
                for r in range(1, world):
                    if store.check([f"{key}/fail/{r}"]):
                        why = store.get(f"{key}/fail/{r}").decode()
                        child.kill()
                        break
            time.sleep(0.2)
        if decision == "done":
            # the line is out; let the child finish its teardown, but not forever
            t_end = time.monotonic() + stall_s
            while child.poll() is None and time.monotonic() < t_end:
                time.sleep(0.2)
            child.kill()
            return 0
        child.kill()
        if decision.startswith("fail"):
            print(f"bench supervisor: attempt {a} ({name}) failed: {decision[5:]}", file=sys.stderr, flush=True)
            return 1
        reason = f"attempt {a} ({name} combines) ended: {decision.split(':', 1)[1]}"
        print(f"bench supervisor: {reason}; starting attempt {a + 1} ({attempts[a + 1][0]} combines)",
              file=sys.stderr, flush=True)
    return 1
