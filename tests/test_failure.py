import threading
import time

from simple_distributed_machine_learning_amd.utils.failure import Heartbeat


class FakeStore:
    def __init__(self):
        self.d, self.lock = {}, threading.Lock()

    def set(self, k, v):
        with self.lock:
            self.d[k] = v.encode() if isinstance(v, str) else v

    def get(self, k):
        with self.lock:
            return self.d[k]

    def check(self, keys):
        with self.lock:
            return all(k in self.d for k in keys)


def test_heartbeat_detects_silent_peer():
    store = FakeStore()
    failed = []
    hb0 = Heartbeat(0, [0, 1], interval_s=0.05, timeout_s=0.3, store=store,
                    on_failure=lambda p, age: failed.append(p)).start()
    hb1 = Heartbeat(1, [0, 1], interval_s=0.05, timeout_s=0.3, store=store,
                    on_failure=lambda p, age: None).start()
    time.sleep(0.5)
    assert not failed  # both alive
    hb1.stop(clean=False)  # peer 1 dies
    t0 = time.time()
    while not failed and time.time() - t0 < 3:
        time.sleep(0.05)
    hb0.stop()
    assert failed == [1]


def test_heartbeat_never_started_peer():
    store = FakeStore()
    failed = []
    hb = Heartbeat(0, [0, 1], interval_s=0.05, timeout_s=0.2, store=store,
                   on_failure=lambda p, age: failed.append(p)).start()
    t0 = time.time()
    while not failed and time.time() - t0 < 3:
        time.sleep(0.05)
    hb.stop()
    assert failed == [1]


def test_heartbeat_clean_exit_is_not_a_failure():
    """A peer that finished (stop() publishes hb/<rank>=done) stays 'alive' for a slower rank."""
    store = FakeStore()
    failed = []
    hb0 = Heartbeat(0, [0, 1], interval_s=0.05, timeout_s=0.2, store=store,
                    on_failure=lambda p, age: failed.append(p)).start()
    hb1 = Heartbeat(1, [0, 1], interval_s=0.05, timeout_s=0.2, store=store,
                    on_failure=lambda p, age: None).start()
    time.sleep(0.2)
    hb1.stop()  # clean finish
    time.sleep(0.8)  # well past timeout_s
    hb0.stop()
    assert failed == []
