"""Failure detection: peer heartbeats over the rendezvous store.

The reference disables every timeout (``rpc_timeout=0`` / ``timeout=0``,
/root/reference/simple_distributed.py:36, :167): a dead peer hangs the job forever
(SURVEY.md §5). Here, besides finite process-group timeouts (parallel/mesh.py), each rank
runs a tiny daemon thread that publishes ``hb/<rank> = <unix time>`` to the TCPStore and
checks its peers; if a peer goes silent for ``timeout_s`` the rank reports it and exits
non-zero instead of hanging in a collective.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Optional, Sequence

import torch.distributed as dist


DONE = "done"


class Heartbeat:
    def __init__(self, rank: int, peers: Sequence[int], interval_s: float = 2.0, timeout_s: float = 60.0,
                 store=None, on_failure: Optional[Callable[[int, float], None]] = None):
        self.rank, self.peers = rank, [p for p in peers if p != rank]
        self.interval_s, self.timeout_s = interval_s, timeout_s
        self.store = store if store is not None else _default_store()
        self.on_failure = on_failure or _exit_on_failure
        self._stop = threading.Event()
        self._clean = False
        self._done_sent = False
        self._thread = None
        self.failed_peer = None

    def start(self):
        if self.store is None:
            return self
        self._beat()
        self._thread = threading.Thread(target=self._loop, name="sdml-heartbeat", daemon=True)
        self._thread.start()
        return self

    def _beat(self):
        self.store.set(f"hb/{self.rank}", repr(time.time()))

    def _loop(self):
        try:
            self._watch()
        finally:
            # the clean-exit marker comes from THIS thread, after its last beat: a beat still in flight
            # can no longer land after it and make a finished rank look alive-but-stale
            if self._stop.is_set() and self._clean:
                self._publish_done()

    def _publish_done(self):
        self._done_sent = True
        try:
            self.store.set(f"hb/{self.rank}", DONE)
        except Exception:  # noqa: BLE001  store already torn down
            pass

    def _watch(self):
        t_start = time.time()
        while not self._stop.wait(self.interval_s):
            try:
                self._beat()
                now = time.time()
                for p in self.peers:
                    key = f"hb/{p}"
                    try:
                        if not self.store.check([key]):
                            if now - t_start > self.timeout_s:
                                self._fail(p, now - t_start)
                                return
                            continue
                        val = self.store.get(key).decode()
                        if val == DONE:  # the peer finished cleanly: never a failure
                            continue
                        last = float(val)
                    except Exception:  # noqa: BLE001  store gone: master died
                        self._fail(p, -1.0)
                        return
                    if now - last > self.timeout_s:
                        self._fail(p, now - last)
                        return
            except Exception:  # noqa: BLE001
                if self._stop.is_set():
                    return
                self._fail(-1, -1.0)
                return

    def _fail(self, peer: int, age: float):
        if self._stop.is_set():
            return
        self.failed_peer = peer
        self.on_failure(peer, age)

    def stop(self, clean: bool = True):
        """Stop beating. ``clean`` publishes ``hb/<rank> = done`` afterwards, so a slower peer
        (e.g. one still writing its checkpoint) does not read this rank's silence as death."""
        self._clean = clean
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=max(10.0, self.interval_s * 4))
            if not self._thread.is_alive() and (self._done_sent or not clean):
                return  # the thread published the marker (if clean) as its last action
        if clean and self.store is not None and not self._done_sent:  # no thread / stuck / exited early
            self._publish_done()


def _default_store():
    if not dist.is_initialized():
        return None
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001
        return None


def _exit_on_failure(peer: int, age: float):
    sys.stderr.write(f"[sdml] peer failure detected: rank {peer} silent for {age:.1f}s — aborting\n")
    sys.stderr.flush()
    os._exit(17)
