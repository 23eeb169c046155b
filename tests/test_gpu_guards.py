"""Guards around the int8 candidate pass's exactness ("what's weak" #2).

* The first search of a FRESH process, for every int8 kernel family: (I8, I8X3) x (cosine, L2)
  x (query block in LDS or from global memory), at the D of the failing round-3 case (96) and
  at C2's 768.  The round-3 failure -- wrong, certified L2 results -- appeared only on a cold
  first search (the loads still in flight when the compiler copied their registers), so each
  case runs in its own process (tests/_first_search_case.py).
* The finish kernel's approx-vs-exact consistency guard: a planted stale L2 start value (the
  operand class of the round-3 failure) makes the query flagged, not certified.
* The int8 pass's checksum (its H / L accumulator sums against the column sums of the stored
  operands): a planted UNDER-scoring corpus operand, which the guard above cannot see, is flagged.
* A device-memory search queued on a side stream while an add re-derives the int8 setup
  (the add must wait for it).

The contract all three protect is the reference's ranking,
/root/reference/service/optimized_vector_store.py:176-183 (argsort of the exact scores).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def vdb():
    from service import _vdb
    assert _vdb.device_count() >= 1, "no GPU visible"
    return _vdb


CASES = [(p, m, q, D) for D in (96, 768) for p in ("i8", "i8x3") for m in ("cosine", "euclidean")
         for q in (-1, 0)]


@pytest.mark.parametrize("precision,metric,qlds,D", CASES,
                         ids=[f"{p}-{m}-qlds{q}-D{D}" for p, m, q, D in CASES])
def test_first_search_in_a_fresh_process(precision, metric, qlds, D):
    r = subprocess.run([sys.executable, os.path.join(HERE, "_first_search_case.py"), precision, metric, str(qlds),
                        str(D)], capture_output=True, text=True, timeout=110)
    print(r.stdout.strip())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "FIRST OK" in r.stdout


@pytest.fixture
def debug_knobs(monkeypatch):
    """The test-only corruption knobs (debug_*) are refused unless VDB_DEBUG_KNOBS=1."""
    monkeypatch.setenv("VDB_DEBUG_KNOBS", "1")


def test_debug_knobs_refused_without_opt_in(vdb, monkeypatch):
    monkeypatch.delenv("VDB_DEBUG_KNOBS", raising=False)
    ix = vdb.NativeIndex(32, "euclidean")
    ix.add(np.random.default_rng(3).random((100, 32), dtype=np.float32))
    with pytest.raises(Exception, match="test-only"):
        ix.set_param("debug_stale_rinit", 5)
    with pytest.raises(Exception, match="test-only"):
        ix.set_param("debug_sink_row8", 5)


@pytest.mark.parametrize("precision", ["i8", "i8x3", "bf16x3"])
def test_consistency_guard_flags_a_planted_stale_operand(vdb, precision, debug_knobs):
    """A row whose L2 start value is stale (-|x|^2/2 read as 0) over-scores by |x|^2 in the
    candidate pass.  It lands in the rerank set, where its exact key disagrees with its
    approximate score by far more than eps: the finish flags the query (exact path) instead of
    certifying it.  Without the plant the same search certifies every query."""
    rng = np.random.default_rng(41)
    N, D, B, k = 20000, 96, 16, 10
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
    ix = vdb.NativeIndex(D, "euclidean", precision=precision)
    ix.add(V)
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    assert ix.stat("inconsistent_queries") == 0
    f0 = ix.stat("fallback_queries")
    # plant: the row nearest to query 0 after its true top k -- any row works, since a
    # start value of 0 lifts it above every honest score
    ix.set_param("debug_stale_rinit", int(ei[0, -1]) + 1 if ei[0, -1] + 1 < N else 0)
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)  # exact: the exact path rewrote the flagged queries
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("inconsistent_queries") >= 1
    assert ix.stat("fallback_queries") > f0


@pytest.mark.parametrize("precision", ["i8", "i8x3"])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_checksum_flags_a_planted_under_scoring_operand(vdb, precision, metric, debug_knobs):
    """the blind side of the approx-vs-exact guard.  Each query's true top-1
    row has its int8 planes set to -127 (debug_sink_row8: the column sums stay, as for a corpus
    operand the pass reads wrong), so the pass UNDER-scores it for every query (the data are
    non-negative): it never becomes a candidate of any query, and
    the finish's consistency check -- which sees only the rerank set -- has nothing to compare.
    With the pass's checksum off the search returns wrong, certified results (the blind side,
    shown); with it on (the default) every query's H (L) accumulator sums disagree with the
    operands' column sums, every query is flagged, and the exact path returns exact results."""
    rng = np.random.default_rng(43)
    N, D, B, k = 20000, 96, 16, 10
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
    ix = vdb.NativeIndex(D, metric, precision=precision)
    ix.add(V)
    _, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    assert ix.stat("inconsistent_queries") == 0
    for r in sorted(set(ei[:, 0].tolist())):
        ix.set_param("debug_sink_row8", int(r))
    ix.set_param("scan_checksum", 0)
    f0 = ix.stat("fallback_queries")
    _, i, kk = ix.search(Q, k, with_keys=True)
    wrong = int((i != ei).any(axis=1).sum())
    print(f"{precision} {metric}: checksum off -> {wrong} of {B} queries wrong, "
          f"{ix.stat('inconsistent_queries')} flagged inconsistent")
    assert wrong >= 1 and ix.stat("inconsistent_queries") == 0  # nothing else sees it
    ix.set_param("scan_checksum", 1)
    _, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("inconsistent_queries") == B, ix.stat("inconsistent_queries")
    assert ix.stat("fallback_queries") - f0 >= B


def test_add_waits_for_queued_device_search_before_rederiving(vdb):
    """while the int8 setup still comes from few rows, an add re-derives it
    and rebuilds the int8 copy of the rows already there.  A device-memory search queued on a
    side stream just before must finish on the old setup (the add waits for it): both the
    search before and a search after the add are exact."""
    import torch
    rng = np.random.default_rng(43)
    D, k = 128, 10
    V1 = rng.random((3000, D), dtype=np.float32)
    V2 = (rng.random((5000, D), dtype=np.float32) * 2.0 - 0.5).astype(np.float32)  # shifts mu and s_x
    Q = rng.random((64, D), dtype=np.float32)
    for metric in ("cosine", "euclidean"):
        ix = vdb.NativeIndex(D, metric, precision="i8")
        ix.add(V1)
        qd = torch.from_numpy(Q).cuda()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        outs = []
        for _ in range(4):  # several batches in flight on the side stream
            sd = torch.empty((64, k), dtype=torch.float32, device="cuda")
            idd = torch.empty((64, k), dtype=torch.int64, device="cuda")
            kd = torch.empty((64, k), dtype=torch.float64, device="cuda")
            ix.search_device(qd.data_ptr(), 64, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=st.cuda_stream)
            outs.append((idd, kd))
        ix.add(V2)  # 8000 >= 2 x 3000 rows: re-derives mu / s_x / dir and rebuilds Xq[0, 3000)
        torch.cuda.synchronize()
        _, ei, ek = ref_cpu.exact_search(Q, V1, k, metric)
        for idd, kd in outs:
            np.testing.assert_array_equal(idd.cpu().numpy(), ei, err_msg=metric)
            np.testing.assert_array_equal(kd.cpu().numpy(), ek, err_msg=metric)
        s, i, kk = ix.search(Q, k, with_keys=True)
        _, ei2, ek2 = ref_cpu.exact_search(Q, np.concatenate([V1, V2]), k, metric)
        np.testing.assert_array_equal(i, ei2, err_msg=metric)
        np.testing.assert_array_equal(kk, ek2, err_msg=metric)
        ix.close()
