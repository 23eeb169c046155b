"""The store's query coalescer (service/optimized_vector_store.py _QueryCoalescer): concurrent
single-vector queries -- the reference's REST executor runs 4 at a time
(/root/reference/api/routes/vectors.py:43, :226-234) -- join one batched search; each caller
gets its own row, truncated to its own k.  Host logic only (a fake batched search)."""
import threading
import time

import numpy as np
import pytest

from service.optimized_vector_store import _QueryCoalescer


def _fake_search(calls, delay=0.01):
    def run(Q, k):
        calls.append((Q.shape[0], k))
        time.sleep(delay)  # a device scan: other callers arrive meanwhile
        out = []
        for q in Q:
            base = int(q[0])
            ix = [base * 100 + j for j in range(k)]
            out.append((ix, [float(-j) for j in range(k)], [{"id": i} for i in ix]))
        return out
    return run


def test_each_caller_gets_its_row_and_k():
    calls = []
    co = _QueryCoalescer(_fake_search(calls))
    res = {}

    def worker(t):
        for r in range(20):
            q = np.array([t * 1000 + r, 0.0], np.float32)
            k = 1 + (t + r) % 7
            res[(t, r)] = (q, k, co.query(q, k))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for (t, r), (q, k, (ix, sc, md)) in res.items():
        base = int(q[0])
        assert ix == [base * 100 + j for j in range(k)]
        assert sc == [float(-j) for j in range(k)] and len(md) == k
    assert co.queries == 80
    assert co.batches < 80  # concurrent callers shared scans
    assert max(b for b, _ in calls) > 1


def test_alone_runs_at_once_and_errors_reach_every_caller():
    calls = []
    co = _QueryCoalescer(_fake_search(calls, delay=0.0))
    ix, _, _ = co.query(np.array([3, 0], np.float32), 2)
    assert ix == [300, 301] and calls == [(1, 2)]

    def boom(Q, k):
        time.sleep(0.01)
        raise ValueError("device said no")
    co2 = _QueryCoalescer(boom)
    errs = []

    def worker():
        try:
            co2.query(np.zeros(2, np.float32), 1)
        except ValueError as e:
            errs.append(str(e))
    ths = [threading.Thread(target=worker) for _ in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert errs == ["device said no"] * 4
    # the coalescer is usable again after a failure
    co2._run = _fake_search([], 0.0)
    assert co2.query(np.array([1, 0], np.float32), 1)[0] == [100]


@pytest.mark.parametrize("max_batch", [1, 3])
def test_max_batch(max_batch):
    calls = []
    co = _QueryCoalescer(_fake_search(calls), max_batch=max_batch)
    ths = [threading.Thread(target=lambda t=t: co.query(np.array([t, 0], np.float32), 1)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert co.queries == 8 and max(b for b, _ in calls) <= max_batch


def test_linger_gathers_the_wave_and_a_lone_caller_never_waits():
    """Adaptive linger: after batches of 4, a leader that finds 1 pending query waits (up to the
    linger) for the rest of the wave; a caller alone (recent batches of 1) runs at once."""
    calls = []
    co = _QueryCoalescer(_fake_search(calls, delay=0.002), max_inflight=1, linger_us=200_000)
    t0 = time.perf_counter()
    for r in range(3):  # alone: no linger, whatever its length
        assert co.query(np.array([r, 0], np.float32), 1)[0] == [r * 100]
    assert time.perf_counter() - t0 < 0.15 and [b for b, _ in calls] == [1, 1, 1]
    co._recent.extend([4] * 8)  # as after waves of 4 callers
    res = {}

    def worker(t, delay):
        time.sleep(delay)
        res[t] = co.query(np.array([10 + t, 0], np.float32), 2)[0]
    ths = [threading.Thread(target=worker, args=(t, 0.01 * t)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert res == {t: [(10 + t) * 100, (10 + t) * 100 + 1] for t in range(4)}
    assert calls[3:] == [(4, 2)]  # the staggered wave ran as one batch


@pytest.mark.parametrize("inflight,linger", [(1, 0), (2, 0), (2, 300), (3, 50)])
def test_many_callers_every_slot_returns(inflight, linger):
    """8 callers x 40 queries, mixed k classes (k <= 16 / <= 200 / larger), a search of random
    length: every caller gets its own answer, and the leadership slots all come back (nothing is
    left running or pending)."""
    rng = np.random.default_rng(inflight * 1000 + linger)
    delays = iter(rng.random(10_000) * 2e-3)
    calls = []

    def run(Q, k):
        calls.append((Q.shape[0], k))
        time.sleep(next(delays))
        return [([int(q[0]) * 1000 + j for j in range(k)], [0.0] * k, [{}] * k) for q in Q]
    co = _QueryCoalescer(run, max_batch=5, max_inflight=inflight, linger_us=linger)
    bad = []

    def worker(t):
        for r in range(40):
            key = t * 100 + r
            k = [3, 40, 250][(t + r) % 3]
            ix, _, _ = co.query(np.array([key, 0], np.float32), k)
            if ix != [key * 1000 + j for j in range(k)]:
                bad.append((t, r))
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=60)
    assert not any(th.is_alive() for th in ths)
    assert bad == [] and co.queries == 320
    assert co._running == 0 and co._pending == []
    assert max(b for b, _ in calls) <= 5
