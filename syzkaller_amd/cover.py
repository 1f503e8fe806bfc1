"""Host-side mirror of syzkaller's pkg/cover API and the fuzzer/manager signal
loops, running on the MI355X through libsyzsig.so.

Names, argument meaning and results follow the reference
(pkg/cover/cover.go:11-182, syz-fuzzer/fuzzer.go:467-489 and :645-693,
syz-manager/manager.go:769-784, :907-912, :949-956) so the parity tests read
like pkg/cover/cover_test.go.  Arrays are numpy uint32 (PCs / signal).  A Go
`map[uint32]struct{}` is a SignalSet (a 2^32-bit bitmap in HBM).

Empty results are returned as empty arrays (Go returns nil; callers only use
len, and cover_test.go:54 treats two empty results as equal).
"""
import ctypes
from ctypes import byref, c_double, c_int, c_int64, c_size_t, c_uint64, c_void_p

import numpy as np

from . import _lib
from ._lib import call, lib

U32 = np.uint32
U64 = np.uint64


def _p32(a):
    return a.ctypes.data_as(_lib.P32)


def _p64(a):
    return a.ctypes.data_as(_lib.P64)


def _p8(a):
    return a.ctypes.data_as(_lib.P8)


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=U32).reshape(-1))


def _u64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=U64).reshape(-1))


class Context:
    """One HIP stream on one MI355X plus the device memory it owns."""

    def __init__(self, device=0):
        h = c_void_p()
        call("sg_ctx_create", device, byref(h))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib.sg_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        call("sg_ctx_sync", self.h)

    def set_stream(self, hip_stream):
        """Queue on `hip_stream` (an int handle; 0 = the legacy default stream)."""
        call("sg_ctx_set_stream", self.h, c_void_p(hip_stream))

    def reset_stream(self):
        call("sg_ctx_reset_stream", self.h)

    def timing(self, enable):
        call("sg_ctx_timing", self.h, 1 if enable else 0)

    def counter(self, name):
        """sg_ctx_counter: "owner_resets", "owner_floor", "owner_key_space", "max_launch_records",
        the host ingest's "host_copy_bytes" / "host_copy_ns" / "host_wait_ns" / "host_copy_threads",
        "cpu_quota_milli"."""
        v = c_uint64()
        call("sg_ctx_counter", self.h, name.encode(), byref(v))
        return v.value

    def set_option(self, key, value):
        """sg_ctx_set_option: force a path for a test or a measurement (include/syzsig.h lists the keys)."""
        call("sg_ctx_set_option", self.h, key.encode(), int(value))

    def get_option(self, key):
        v = c_int64()
        call("sg_ctx_get_option", self.h, key.encode(), byref(v))
        return v.value

    def kernel_time(self, name):
        ms = c_double()
        n = c_uint64()
        call("sg_ctx_kernel_time", self.h, name.encode(), byref(ms), byref(n))
        return ms.value, n.value


_default = None


def default_context():
    global _default
    if _default is None:
        _default = Context(0)
    return _default


def _ctx(ctx):
    return ctx if ctx is not None else default_context()


class SignalSet:
    """map[uint32]struct{} (syz-fuzzer/fuzzer.go:65-68, syz-manager/manager.go:71-73)."""

    def __init__(self, ctx=None):
        self.ctx = _ctx(ctx)
        h = c_void_p()
        call("sg_set_create", self.ctx.h, byref(h))
        self.h = h

    def close(self):
        if self.h:
            lib.sg_set_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        n = c_uint64()
        call("sg_set_count", self.h, byref(n))
        return n.value

    def clear(self):
        call("sg_set_clear", self.h)

    def export(self):
        n = c_size_t()
        call("sg_set_export", self.h, None, 0, byref(n))
        out = np.empty(n.value, dtype=U32)
        if n.value:
            call("sg_set_export", self.h, _p32(out), out.size, byref(n))
        return out

    def device_words(self):
        return lib.sg_set_device_words(self.h)

    def or_device(self, ptr):
        call("sg_set_or_dev", self.h, c_void_p(ptr))


# ---- pkg/cover/cover.go:160-182 -------------------------------------------------
def SignalNew(base, signal):
    s = _u32(signal)
    out = c_int()
    call("sg_set_new", base.h, _p32(s), s.size, byref(out))
    return bool(out.value)


def SignalDiff(base, signal):
    s = _u32(signal)
    out = np.empty(s.size, dtype=U32)
    n = c_size_t()
    call("sg_set_diff", base.h, _p32(s), s.size, _p32(out), byref(n))
    return out[: n.value]


def SignalAdd(base, signal):
    s = _u32(signal)
    call("sg_set_add", base.h, _p32(s), s.size)


# ---- pkg/cover/cover.go:28-117 --------------------------------------------------
def Canonicalize(cov, ctx=None):
    """In place on a uint32 numpy array (like Go's slice); returns cov[:n]."""
    if not (isinstance(cov, np.ndarray) and cov.dtype == U32 and cov.flags.c_contiguous):
        cov = _u32(cov)
    n = c_size_t()
    call("sg_canonicalize", _ctx(ctx).h, _p32(cov), cov.size, byref(n))
    return cov[: n.value]


def _merge(op, a, b, ctx):
    a, b = _u32(a), _u32(b)
    out = np.empty(a.size + b.size, dtype=U32)
    n = c_size_t()
    call("sg_merge", _ctx(ctx).h, op, _p32(a), a.size, _p32(b), b.size, _p32(out), byref(n))
    return out[: n.value]


def Difference(cov0, cov1, ctx=None):
    return _merge(_lib.OP_DIFFERENCE, cov0, cov1, ctx)


def SymmetricDifference(cov0, cov1, ctx=None):
    return _merge(_lib.OP_SYMDIFF, cov0, cov1, ctx)


def Union(cov0, cov1, ctx=None):
    return _merge(_lib.OP_UNION, cov0, cov1, ctx)


def Intersection(cov0, cov1, ctx=None):
    return _merge(_lib.OP_INTERSECT, cov0, cov1, ctx)


def union_fold(vals, off, group=None, ngroups=1, ctx=None):
    """The manager's cover.Union folds (syz-manager/html.go:84/:94/:184/:306,
    manager.go:916-917) for every group at once.  Returns (vals, off) with one
    fold per group."""
    vals, off = _u32(vals), _u64(off)
    n = off.size - 1
    g = _u32(group) if group is not None else None
    out = np.empty(max(vals.size, 1), dtype=U32)
    oo = np.zeros(ngroups + 1, dtype=U64)
    call("sg_union_fold", _ctx(ctx).h, _p32(vals), _p64(off), n, _p32(g) if g is not None else None, ngroups,
         _p32(out), out.size, _p64(oo))
    return out[: int(oo[-1])].copy(), oo


def HasDifference(cov0, cov1, ctx=None):
    a, b = _u32(cov0), _u32(cov1)
    out = c_int()
    call("sg_has_difference", _ctx(ctx).h, _p32(a), a.size, _p32(b), b.size, byref(out))
    return bool(out.value)


def has_difference_batch(a, a_beg, a_len, b, b_beg, b_len, ctx=None):
    """HasDifference (cover.go:106-117) of every pair, laid out as merge_batch's:
    a bool array."""
    a, b = _u32(a), _u32(b)
    ab, al, bb, bl = _u64(a_beg), _u64(a_len), _u64(b_beg), _u64(b_len)
    out = np.zeros(max(ab.size, 1), dtype=np.uint8)
    call("sg_has_difference_batch", _ctx(ctx).h, _p32(a), a.size, _p64(ab), _p64(al), _p32(b), b.size, _p64(bb),
         _p64(bl), ab.size, out.ctypes.data)
    return out[: ab.size].astype(bool)


def to_csr(lists):
    lens = np.array([len(x) for x in lists], dtype=U64)
    off = np.zeros(len(lists) + 1, dtype=U64)
    np.cumsum(lens, out=off[1:])
    vals = np.concatenate([_u32(x) for x in lists]) if lists else np.empty(0, dtype=U32)
    return _u32(vals), off


def minimize_order(off):
    off = _u64(off)
    n = off.size - 1
    order = np.empty(n, dtype=U32)
    call("sg_minimize_order", _p64(off), n, _p32(order))
    return order


def minimize_csr(vals, off, order=None, ctx=None):
    vals, off = _u32(vals), _u64(off)
    n = off.size - 1
    order = minimize_order(off) if order is None else _u32(order)
    out = np.empty(n, dtype=U32)
    m = c_size_t()
    call("sg_minimize", _ctx(ctx).h, _p32(vals), _p64(off), n, _p32(order), _p32(out), byref(m))
    return out[: m.value]


def Minimize(corpus, ctx=None):
    """pkg/cover/cover.go:120-146, including its sort.Sort order."""
    vals, off = to_csr(corpus)
    return [int(i) for i in minimize_csr(vals, off, None, ctx)]


# ---- batched hot path -------------------------------------------------------------
def triage_batch(maxset, newset, vals, rec_off, want_diff=True, ctx=None):
    """syz-fuzzer/fuzzer.go:645-693 over a batch of call records.

    Returns (rec_new uint8[nrec], diff_vals, diff_off) -- diff_* None if not
    requested."""
    vals, off = _u32(vals), _u64(rec_off)
    nrec = off.size - 1
    rec_new = np.zeros(nrec, dtype=np.uint8)
    c = maxset.ctx if ctx is None else ctx
    if want_diff:
        dv = np.empty(max(vals.size, 1), dtype=U32)
        do = np.empty(nrec + 1, dtype=U64)
        nd = c_uint64()
        call("sg_triage_batch", c.h, maxset.h, newset.h if newset is not None else None, _p32(vals), _p64(off), nrec,
             _p8(rec_new), _p32(dv), _p64(do), byref(nd))
        return rec_new, dv[: nd.value], do
    call("sg_triage_batch", c.h, maxset.h, newset.h if newset is not None else None, _p32(vals), _p64(off), nrec, _p8(rec_new),
         None, None, None)
    return rec_new, None, None


def triage_traces(maxset, newset, pcs, call_off, ctx=None):
    """fuzzer.go:645-693 over a batch given as raw per-call PC traces (set-exact
    edge signal, executor.h:389-401): the per-call flags, sets updated."""
    p, off = _u32(pcs), _u64(call_off)
    ncalls = off.size - 1
    rec_new = np.zeros(ncalls, dtype=np.uint8)
    c = maxset.ctx if ctx is None else ctx
    call("sg_triage_traces", c.h, maxset.h, newset.h if newset is not None else None, _p32(p), _p64(off), ncalls,
         _p8(rec_new))
    return rec_new


def triage_traces_queued(maxset, newset, pcs, call_off, prog_off, ctx=None):
    """The fuzzer's step from raw traces (sg_triage_traces_queued): the
    per-call flags of fuzzer.go:645-693 (sets updated, set-exact) and the
    executor-exact signal list of every queued call (fuzzer.go:678-683;
    executor.h:389-401), empty for the others.  Returns (rec_new, vals, off)."""
    p, co, po = _u32(pcs), _u64(call_off), _u64(prog_off)
    ncalls = co.size - 1
    rec_new = np.zeros(max(ncalls, 1), dtype=np.uint8)
    sv = np.empty(max(p.size, 1), dtype=U32)
    so = np.empty(ncalls + 1, dtype=U64)
    c = maxset.ctx if ctx is None else ctx
    call("sg_triage_traces_queued", c.h, maxset.h, newset.h if newset is not None else None, _p32(p), _p64(co),
         _p64(po), po.size - 1, _p8(rec_new), _p32(sv), _p64(so))
    return rec_new[:ncalls], sv[: int(so[-1])], so


def add_inputs(corpus, maxset, vals, off, ctx=None):
    """syz-fuzzer/fuzzer.go:467-489 addInput over a batch of inputs."""
    vals, off = _u32(vals), _u64(off)
    c = corpus.ctx if ctx is None else ctx
    call("sg_add_inputs", c.h, corpus.h, maxset.h, _p32(vals), _p64(off), off.size - 1)


def triage_newsig(corpus, vals, off, ctx=None):
    """syz-fuzzer/fuzzer.go:526-532 over a batch of triage inputs:
    new_k = Canonicalize(SignalDiff(corpusSignal, S_k)).  Returns (vals, off)."""
    vals, off = _u32(vals), _u64(off)
    n = off.size - 1
    nv = np.empty(max(vals.size, 1), dtype=U32)
    no = np.zeros(n + 1, dtype=U64)
    c = corpus.ctx if ctx is None else ctx
    call("sg_triage_newsig", c.h, corpus.h, _p32(vals), _p64(off), n, _p32(nv), _p64(no))
    return nv[: int(no[-1])], no


def triage_intersect(new_vals, new_off, r_vals, r_off, ctx=None):
    """fuzzer.go:567 over a batch: new_k = Intersection(new_k, Canonicalize(R_k)).
    Returns the packed (vals, off)."""
    nv, no = _u32(new_vals).copy(), _u64(new_off)
    rv, ro = _u32(r_vals), _u64(r_off)
    n = no.size - 1
    lens = np.zeros(n, dtype=U64)
    call("sg_triage_intersect", _ctx(ctx).h, _p32(nv), _p64(no), _p32(rv), _p64(ro), n, _p64(lens))
    out_off = np.concatenate([[0], np.cumsum(lens)]).astype(U64)
    out = np.concatenate([nv[int(no[k]): int(no[k]) + int(lens[k])] for k in range(n)]) if n else nv[:0]
    return out.astype(U32), out_off


def triage_subset(new_vals, new_off, r_vals, r_off, ctx=None):
    """fuzzer.go:584-587, the minimisation predicate over a batch:
    ok[k] = len(Intersection(new_k, Canonicalize(R_k))) == len(new_k)."""
    nv, no = _u32(new_vals), _u64(new_off)
    rv, ro = _u32(r_vals), _u64(r_off)
    n = no.size - 1
    ok = np.zeros(n, dtype=np.uint8)
    call("sg_triage_subset", _ctx(ctx).h, _p32(nv), _p64(no), _p32(rv), _p64(ro), n, _p8(ok))
    return ok


def accept_batch(corpus_sig, corpus_cov, sig_vals, sig_off, cov_vals=None, cov_off=None, ctx=None):
    """syz-manager/manager.go:907-912 NewInput acceptance over a batch."""
    sv, so = _u32(sig_vals), _u64(sig_off)
    n = so.size - 1
    acc = np.zeros(n, dtype=np.uint8)
    c = corpus_sig.ctx if ctx is None else ctx
    if corpus_cov is not None and cov_vals is not None:
        cv, co = _u32(cov_vals), _u64(cov_off)
        call("sg_accept_batch", c.h, corpus_sig.h, corpus_cov.h, _p32(sv), _p64(so), _p32(cv), _p64(co), n, _p8(acc))
    else:
        call("sg_accept_batch", c.h, corpus_sig.h, None, _p32(sv), _p64(so), None, None, n, _p8(acc))
    return acc


def merge_poll(mgr_max, a_vals, a_off, ctx=None):
    """syz-manager/manager.go:949-956 over polls in arrival order."""
    av, ao = _u32(a_vals), _u64(a_off)
    npoll = ao.size - 1
    nv = np.empty(max(av.size, 1), dtype=U32)
    no = np.empty(npoll + 1, dtype=U64)
    c = mgr_max.ctx if ctx is None else ctx
    call("sg_merge_poll", c.h, mgr_max.h, _p32(av), _p64(ao), npoll, _p32(nv), _p64(no))
    return nv[: int(no[-1])], no


# ---- RPC payloads (pkg/rpctype/rpctype.go:8-63) ------------------------------------
def delta_encode(vals, off, ctx=None):
    """Sorted lists -> their delta-varint payloads (bytes, byte offsets)."""
    vals, off = _u32(vals), _u64(off)
    n = off.size - 1
    bo = np.zeros(n + 1, dtype=U64)
    out = np.empty(max(5 * vals.size, 1), dtype=np.uint8)
    call("sg_delta_encode_batch", _ctx(ctx).h, _p32(vals), _p64(off), n, _p8(out), out.size, _p64(bo))
    return out[: int(bo[-1])].copy(), bo


def delta_decode(data, data_off, ctx=None):
    """Payloads -> the sorted lists (vals, off)."""
    data = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                                else np.asarray(data, dtype=np.uint8))
    do = _u64(data_off)
    n = do.size - 1
    vals = np.empty(max(data.size, 1), dtype=U32)
    off = np.zeros(n + 1, dtype=U64)
    call("sg_delta_decode_batch", _ctx(ctx).h, _p8(data), _p64(do), n, _p32(vals), vals.size, _p64(off))
    return vals[: int(off[-1])].copy(), off


def set_encode(sset):
    """The set's members as one payload (PollArgs / ConnectRes / PollRes .MaxSignal)."""
    nb = c_size_t()
    call("sg_set_encode", sset.h, None, 0, byref(nb))
    out = np.empty(max(nb.value, 1), dtype=np.uint8)
    call("sg_set_encode", sset.h, _p8(out), out.size, byref(nb))
    return out[: nb.value].tobytes()


def set_decode_add(sset, payload):
    """SignalAdd of a payload (fuzzer.go:146-151, :392-398); returns its value count."""
    data = np.frombuffer(bytes(payload), dtype=np.uint8).copy()
    cnt = c_uint64()
    call("sg_set_decode_add", sset.h, _p8(data), data.size, byref(cnt))
    return cnt.value


def sancov(cov_vals, cov_off, ctx=None):
    """tools/syz-execprog/execprog.go:159-177 sancov files of a batch of calls (list of bytes)."""
    cv, co = _u32(cov_vals), _u64(cov_off)
    n = co.size - 1
    out = np.empty(max(8 * (n + cv.size), 1), dtype=np.uint8)
    call("sg_sancov_batch", _ctx(ctx).h, _p32(cv), _p64(co), n, _p8(out))
    return [out[8 * (k + int(co[k])): 8 * (k + 1 + int(co[k + 1]))].tobytes() for k in range(n)]


def canonicalize_batch(vals, off, ctx=None):
    """Batched Canonicalize in place; returns per-segment canonical lengths."""
    if not (isinstance(vals, np.ndarray) and vals.dtype == U32 and vals.flags.c_contiguous):
        raise TypeError("canonicalize_batch works in place on a contiguous uint32 array")
    off = _u64(off)
    n = off.size - 1
    lens = np.zeros(n, dtype=U64)
    call("sg_canonicalize_batch", _ctx(ctx).h, _p32(vals), _p64(off), n, _p64(lens))
    return lens


def merge_batch(op, a, a_beg, a_len, b, b_beg, b_len, ctx=None):
    a, b = _u32(a), _u32(b)
    ab, al, bb, bl = _u64(a_beg), _u64(a_len), _u64(b_beg), _u64(b_len)
    npair = ab.size
    ob = np.zeros(npair, dtype=U64)
    if npair > 1:
        np.cumsum(al[:-1] + bl[:-1], out=ob[1:])
    total = int((al + bl).sum())
    out = np.empty(max(total, 1), dtype=U32)
    ol = np.zeros(npair, dtype=U64)
    call("sg_merge_batch", _ctx(ctx).h, op, _p32(a), a.size, _p64(ab), _p64(al), _p32(b), b.size, _p64(bb),
         _p64(bl), npair, _p32(out), out.size, _p64(ob), _p64(ol))
    return [out[int(ob[k]): int(ob[k] + ol[k])] for k in range(npair)]


def exec_signal(pcs, call_off, prog_off, ctx=None):
    """executor/executor.h:389-401 + :497-526 over a batch of programs."""
    p, co, po = _u32(pcs), _u64(call_off), _u64(prog_off)
    ncalls = co.size - 1
    sv = np.empty(max(p.size, 1), dtype=U32)
    so = np.empty(ncalls + 1, dtype=U64)
    call("sg_exec_signal", _ctx(ctx).h, _p32(p), _p64(co), _p64(po), po.size - 1, _p32(sv), _p64(so))
    return sv[: int(so[-1])], so


def cover_uncovered(cov, base, sym_start, sym_end, all_pcs, ctx=None):
    """syz-manager/cover.go:91-103 + uncoveredPcsInFuncs (:257-307); ascending."""
    c, ss, se, ap = _u32(cov), _u64(sym_start), _u64(sym_end), _u64(all_pcs)
    out = np.empty(max(ap.size, 1), dtype=U64)
    n = c_size_t()
    call("sg_cover_uncovered", _ctx(ctx).h, _p32(c), c.size, base, _p64(ss), _p64(se), ss.size, _p64(ap), ap.size,
         _p64(out), byref(n))
    return out[: n.value]


# pkg/ipc/ipc_linux.go:168-307 status codes (include/syzsig.h SG_IPC_*)
IPC_OK, IPC_NO_NCMD, IPC_SHORT_HEADER, IPC_BAD_INDEX, IPC_BAD_CALLNUM, IPC_DOUBLE = 0, 1, 2, 3, 4, 5
IPC_SIGNAL_SIZE, IPC_COVER_SIZE, IPC_COMPS_SHORT, IPC_COMPS_TYPE = 6, 7, 8, 9


def ipc_parse(out, out_off, call_off, call_nums=None, cover=True, ctx=None):
    """readOutCoverage (pkg/ipc/ipc_linux.go:168-307) over a batch of program
    output regions.  Returns (errno int64[nrec], fault u8[nrec], status
    int32[nprog], sig_vals, sig_off, cov_vals, cov_off); cov_* are None when
    cover=False."""
    w, oo, co = _u32(out), _u64(out_off), _u64(call_off)
    nprog = oo.size - 1
    assert co.size == nprog + 1
    nrec = int(co[-1])
    nums = None if call_nums is None else _u32(call_nums)
    assert nums is None or nums.size == nrec
    err = np.empty(max(nrec, 1), dtype=np.int64)
    fault = np.empty(max(nrec, 1), dtype=np.uint8)
    status = np.empty(max(nprog, 1), dtype=np.int32)
    sv = np.empty(max(w.size, 1), dtype=U32)
    so = np.empty(nrec + 1, dtype=U64)
    cv = np.empty(max(w.size, 1), dtype=U32) if cover else None
    cvo = np.empty(nrec + 1, dtype=U64) if cover else None
    call("sg_ipc_parse", _ctx(ctx).h, _p32(w), _p64(oo), _p64(co), _p32(nums) if nums is not None else None, nprog,
         err.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), _p8(fault),
         status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _p64(so), _p32(sv),
         _p64(cvo) if cover else None, _p32(cv) if cover else None)
    return (err[:nrec], fault[:nrec], status[:nprog], sv[: int(so[-1])], so,
            cv[: int(cvo[-1])] if cover else None, cvo)
