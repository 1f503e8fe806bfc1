"""Executor output ingest (pkg/ipc/ipc_linux.go:168-307 readOutCoverage):
the oracle against the writer layout on CPU, then sg_ipc_parse bit-exact
against the oracle on the GPU.  Parity unpinned by reference fixtures (none
exist for this reader; see oracle/ipc_oracle.py)."""
import numpy as np
import pytest

from oracle import ipc_oracle as I
from tests import ipc_cases as K


def test_oracle_round_trip_of_the_writer_layout():
    rng = np.random.default_rng(1)
    calls = [(ci, [int(x) for x in rng.integers(0, 1 << 32, size=10 + ci, dtype=np.uint64)], [0x81000000 + 16 * ci])
             for ci in [2, 0, 1]]
    words = []
    for ci, sig, cov in calls:
        words += I.write_call(ci, 100 + ci, 0xFFFFFFFF if ci == 1 else ci, ci & 1, sig, cov)
    st, info = I.read_out_coverage([3] + words, 4, [100, 101, 102, 103])
    assert st == I.OK
    for ci, sig, cov in calls:
        assert info[ci]["signal"] == sig and info[ci]["cover"] == cov
        assert info[ci]["fault"] == ci & 1
    assert info[1]["errno"] == 0xFFFFFFFF  # int(uint32), not -1
    assert info[3] == dict(errno=-1, fault=0, signal=None, cover=None)  # not executed


def test_oracle_error_paths():
    assert I.read_out_coverage([], 2)[0] == I.NO_NCMD
    assert I.read_out_coverage([1, 0, 0, 0], 2)[0] == I.SHORT_HEADER
    assert I.read_out_coverage([1] + I.write_call(2, 0, 0, 0, [1]), 2)[0] == I.BAD_INDEX
    assert I.read_out_coverage([1] + I.write_call(1, 9, 0, 0, [1]), 2, [0, 8])[0] == I.BAD_CALLNUM
    st, info = I.read_out_coverage([2] + I.write_call(1, 0, 0, 0, []) * 2, 2)
    assert st == I.DOUBLE and info[1]["signal"] == []  # an empty Signal is non-nil
    st, info = I.read_out_coverage([1, 0, 0, 5, 1, 10, 0, 0, 1, 2], 1)
    assert st == I.SIGNAL_SIZE and info[0]["errno"] == 5 and info[0]["signal"] is None
    st, info = I.read_out_coverage([1, 0, 0, 0, 0, 2, 10, 0, 1, 2], 1)
    assert st == I.COVER_SIZE and info[0]["signal"] == [1, 2] and info[0]["cover"] is None
    assert I.read_out_coverage([1, 0, 0, 0, 0, 0, 0, 1, 8], 1)[0] == I.COMPS_TYPE
    assert I.read_out_coverage([1, 0, 0, 0, 0, 0, 0, 1, 6, 1], 1)[0] == I.COMPS_SHORT
    assert I.read_out_coverage([1, 0, 0, 0, 0, 0, 0, 1, 0, 1, 2, 3], 1)[0] == I.COMPS_SHORT
    assert I.read_out_coverage([1, 0, 0, 0, 0, 0, 0, 1, 0, 1, 2, 3, 4], 1)[0] == I.OK


def test_cases_reach_every_error_path():
    out, oo, co, nums = K.batch(3, nprog=240, kinds=K.FAULTS)
    _, _, status, _, _ = I.parse_batch(out, oo, co, nums)
    assert set(status) == set(range(10))


def _check(C, out, oo, co, nums, cover=True):
    err, fault, status, sv, so, cv, cvo = C.ipc_parse(out, oo, co, nums, cover=cover)
    e_err, e_fault, e_status, e_sig, e_cov = I.parse_batch(out, oo, co, nums)
    assert status.tolist() == e_status
    assert err.tolist() == e_err
    assert fault.tolist() == e_fault
    assert np.diff(so.astype(np.int64)).tolist() == [len(s) for s in e_sig]
    assert sv.tolist() == [x for s in e_sig for x in s]
    if cover:
        assert np.diff(cvo.astype(np.int64)).tolist() == [len(c) for c in e_cov]
        assert cv.tolist() == [x for c in e_cov for x in c]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ipc_parse_vs_oracle(ctx, seed):
    from syzkaller_amd import cover as C

    out, oo, co, nums = K.batch(seed, nprog=300)
    _check(C, out, oo, co, nums)
    _check(C, out, oo, co, None, cover=False)  # no call-number check, signal only


@pytest.mark.gpu
def test_ipc_parse_every_error_path_and_edges(ctx):
    from syzkaller_amd import cover as C

    out, oo, co, nums = K.batch(7, nprog=240, kinds=K.FAULTS)
    _check(C, out, oo, co, nums)
    # empty batch, programs with no calls, one long record (> one wave's worth)
    _check(C, np.zeros(0, np.uint32), np.zeros(1, np.uint64), np.zeros(1, np.uint64), None)
    _check(C, np.array([0, 0], np.uint32), np.array([0, 1, 2], np.uint64), np.array([0, 0, 0], np.uint64), None)
    w = [1] + I.write_call(0, 0, 0, 0, list(range(100000)), list(range(5, 70000)))
    _check(C, np.array(w, np.uint32), np.array([0, len(w)], np.uint64), np.array([0, 1], np.uint64), None)


@pytest.mark.gpu
def test_ipc_parse_feeds_triage(ctx):
    """The parsed signal CSR is the triage input as is (fuzzer.go:645-693)."""
    from oracle import pyoracle as O
    from syzkaller_amd import cover as C

    out, oo, co, nums = K.batch(11, nprog=200, kinds=["ok"], maxsig=2000)
    _, _, status, sv, so, _, _ = C.ipc_parse(out, oo, co, nums, cover=False)
    assert (status == 0).all()
    m, n = C.SignalSet(), C.SignalSet()
    flags, _, _ = C.triage_batch(m, n, sv, so)
    om, on = O.OSet(), O.OSet()
    eflags, _, _ = O.triage_batch(om, on, sv, so)
    assert np.array_equal(np.asarray(flags), np.asarray(eflags))


@pytest.mark.gpu
def test_ipc_parse_feeds_triage_with_failed_programs(ctx):
    """A batch with every reader error path planted: the failed programs'
    records carry no signal in the CSR (execute1 never returns their info,
    fuzzer.go:752-768), so triaging the CSR as is equals the oracle's
    sequential loop over the successful programs' records only."""
    from oracle import pyoracle as O
    from syzkaller_amd import cover as C

    out, oo, co, nums = K.batch(13, nprog=240, kinds=K.FAULTS, maxsig=800)
    _, _, status, sv, so, _, _ = C.ipc_parse(out, oo, co, nums, cover=False)
    assert (status != 0).any() and (status == 0).any()
    # the oracle's view: the reader's signal of the successful programs only
    _, _, e_status, e_sig, _ = I.parse_batch(out, oo, co, nums)
    assert status.tolist() == e_status
    ok_recs = [r for p in range(len(e_status)) if e_status[p] == 0 for r in range(int(co[p]), int(co[p + 1]))]
    for p in range(len(e_status)):
        if e_status[p] != 0:
            assert all(so[r + 1] == so[r] for r in range(int(co[p]), int(co[p + 1])))
    m, n = C.SignalSet(), C.SignalSet()
    flags, _, _ = C.triage_batch(m, n, sv, so)
    om, on = O.OSet(), O.OSet()
    ok_sig = [e_sig[r] for r in ok_recs]
    ov = np.array([x for s in ok_sig for x in s], np.uint32)
    oo_ = np.concatenate([[0], np.cumsum([len(s) for s in ok_sig])]).astype(np.uint64)
    eflags, _, _ = O.triage_batch(om, on, ov, oo_)
    assert np.array_equal(np.asarray(flags)[ok_recs], np.asarray(eflags))
    assert not np.asarray(flags)[[r for r in range(flags.size) if r not in set(ok_recs)]].any()
    assert np.array_equal(m.export(), om.export()) and np.array_equal(n.export(), on.export())
