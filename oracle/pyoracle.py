"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end of oracle/libsigoracle.so (the C restatement of the
reference, oracle/sigoracle.c) and of oracle/_ref/libref_executor.so (the
reference executor compiled from its own sources).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this; the
product (syzkaller_amd/) never does.
"""
import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libsigoracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_executor.so")

P32 = POINTER(c_uint32)
P64 = POINTER(c_uint64)
P8 = POINTER(c_uint8)

DIFF, SYMDIFF, UNION, INTER = 0, 1, 2, 3


def build():
    """Compile the oracle (and, where the reference checkout exists, _ref)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load():
    if not os.path.exists(ORACLE_SO):
        build()
    L = ctypes.CDLL(ORACLE_SO)
    sig = {
        "orc_canonicalize": (c_size_t, [P32, c_size_t]),
        "orc_foreach": (c_size_t, [c_int, P32, c_size_t, P32, c_size_t, P32]),
        "orc_has_difference": (c_int, [P32, c_size_t, P32, c_size_t]),
        "orc_set_new": (c_void_p, []),
        "orc_set_free": (None, [c_void_p]),
        "orc_set_count": (c_size_t, [c_void_p]),
        "orc_set_has": (c_int, [c_void_p, c_uint32]),
        "orc_set_export": (c_size_t, [c_void_p, P32]),
        "orc_signal_new": (c_int, [c_void_p, P32, c_size_t]),
        "orc_signal_diff": (c_size_t, [c_void_p, P32, c_size_t, P32]),
        "orc_signal_add": (None, [c_void_p, P32, c_size_t]),
        "orc_triage_batch": (c_uint64, [c_void_p, c_void_p, P32, P64, c_size_t, P8, P32, P64]),
        "orc_triage_procs": (c_int, [c_void_p, c_void_p, P32, P64, P64, c_size_t, c_int, P8]),
        "orc_add_inputs": (None, [c_void_p, c_void_p, P32, P64, c_size_t]),
        "orc_accept_batch": (None, [c_void_p, c_void_p, P32, P64, P32, P64, c_size_t, P8]),
        "orc_merge_poll": (c_uint64, [c_void_p, P32, P64, c_size_t, P32, P64]),
        "orc_minimize_order": (None, [P64, c_size_t, P32]),
        "orc_minimize_ordered": (c_size_t, [P32, P64, c_size_t, P32, P32]),
        "orc_exec_hash": (c_uint32, [c_uint32]),
        "orc_exec_signal_batch": (c_uint64, [P32, P64, P64, c_size_t, P32, P64]),
        "orc_cover_uncovered": (c_size_t, [P32, c_size_t, c_uint32, P64, P64, c_size_t, P64, c_size_t, P64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


L = _load()


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))


def _u64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1))


def p32(a):
    return a.ctypes.data_as(P32)


def p64(a):
    return a.ctypes.data_as(P64)


def p8(a):
    return a.ctypes.data_as(P8)


class OSet:
    """Go map[uint32]struct{} restated (open addressing)."""

    def __init__(self, values=None):
        self.h = L.orc_set_new()
        if values is not None:
            self.add(values)

    def __del__(self):
        if getattr(self, "h", None):
            L.orc_set_free(self.h)
            self.h = None

    def __len__(self):
        return L.orc_set_count(self.h)

    def add(self, values):
        v = _u32(values)
        L.orc_signal_add(self.h, p32(v), v.size)

    def has(self, x):
        return bool(L.orc_set_has(self.h, int(x)))

    def export(self):
        out = np.empty(max(len(self), 1), dtype=np.uint32)
        n = L.orc_set_export(self.h, p32(out))
        return out[:n]


def canonicalize(v):
    a = _u32(v).copy()
    n = L.orc_canonicalize(p32(a), a.size)
    return a, n  # full in-place array (Go semantics) and canonical length


def foreach(op, a, b):
    a, b = _u32(a), _u32(b)
    out = np.empty(a.size + b.size + 1, dtype=np.uint32)
    n = L.orc_foreach(op, p32(a), a.size, p32(b), b.size, p32(out))
    return out[:n].copy()


def has_difference(a, b):
    a, b = _u32(a), _u32(b)
    return bool(L.orc_has_difference(p32(a), a.size, p32(b), b.size))


def signal_new(s, sig):
    v = _u32(sig)
    return bool(L.orc_signal_new(s.h, p32(v), v.size))


def signal_diff(s, sig):
    v = _u32(sig)
    out = np.empty(max(v.size, 1), dtype=np.uint32)
    n = L.orc_signal_diff(s.h, p32(v), v.size, p32(out))
    return out[:n].copy()


def triage_newsig(corpus, vals, off):
    """syz-fuzzer/fuzzer.go:526-532 per input: Canonicalize(SignalDiff(corpusSignal, S_k))
    (cover.go:169-176 then cover.go:28-40), every input against the same corpus."""
    vals, off = _u32(vals), _u64(off)
    outs = []
    for k in range(off.size - 1):
        a, n = canonicalize(signal_diff(corpus, vals[int(off[k]):int(off[k + 1])]))
        outs.append(a[:n])
    return _csr(outs)


def triage_intersect(new_vals, new_off, r_vals, r_off):
    """fuzzer.go:567 per input: Intersection(new_k, Canonicalize(R_k)) (cover.go:72-79)."""
    outs = []
    for k in range(new_off.size - 1):
        r, n = canonicalize(r_vals[int(r_off[k]):int(r_off[k + 1])])
        outs.append(foreach(INTER, new_vals[int(new_off[k]):int(new_off[k + 1])], r[:n]))
    return _csr(outs)


def triage_subset(new_vals, new_off, r_vals, r_off):
    """fuzzer.go:584-587 per input: len(Intersection(new_k, Canonicalize(R_k))) == len(new_k)."""
    iv, io = triage_intersect(new_vals, new_off, r_vals, r_off)
    return ((io[1:] - io[:-1]) == (_u64(new_off)[1:] - _u64(new_off)[:-1])).astype(np.uint8)


def union_fold(vals, off, group=None, ngroups=1):
    """syz-manager/html.go:84/:94/:184/:306: cov = cover.Union(cov, inp.Cover)
    over the inputs of each group, in input order (cover.go:63-70 via foreach)."""
    vals, off = _u32(vals), _u64(off)
    covs = [np.zeros(0, np.uint32) for _ in range(ngroups)]
    for k in range(off.size - 1):
        g = int(group[k]) if group is not None else 0
        covs[g] = foreach(UNION, covs[g], vals[int(off[k]):int(off[k + 1])])
    return _csr(covs)


def put_uvarint(x):
    """Go encoding/binary PutUvarint (LEB128)."""
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def delta_encode_batch(vals, off):
    """delta_encode of every list of a CSR batch at once, vectorised (the same
    bytes as delta_encode list by list; checked against it in
    tests/test_rpc.py): (payload bytes, byte offsets per list)."""
    v = _u32(vals).astype(np.int64)
    o = _u64(off).astype(np.int64)
    prev = np.zeros_like(v)
    prev[1:] = v[:-1]
    lens = np.diff(o)
    prev[o[:-1][lens > 0]] = 0  # each list's first value is encoded whole
    d = v - prev
    assert (d >= 0).all(), "sorted lists"
    nb = np.ones(d.size, np.int64)
    x = d >> 7
    while x.any():  # Uvarint: 7 bits per byte, high bit = more bytes follow
        nb += x > 0
        x >>= 7
    pos = np.cumsum(nb) - nb
    out = np.empty(int(nb.sum()), np.uint8)
    for k in range(int(nb.max()) if nb.size else 0):
        m = nb > k
        out[pos[m] + k] = (((d[m] >> (7 * k)) & 0x7F) | ((nb[m] > k + 1) << 7)).astype(np.uint8)
    cb = np.concatenate([[0], np.cumsum(nb)])
    return out, cb[o].astype(np.uint64)


def delta_encode(lst):
    """The RPC payload of a sorted []uint32 (pkg/rpctype/rpctype.go:8-63 fields):
    PutUvarint of the first value, then of each successive difference."""
    out, prev = bytearray(), 0
    for v in lst:
        v = int(v)
        assert v >= prev, "sorted input"
        out += put_uvarint(v - prev)
        prev = v
    return bytes(out)


def delta_decode(data):
    """binary.Uvarint + running sum; ValueError on a malformed payload."""
    vals, x, shift, prev = [], 0, 0, 0
    for i, c in enumerate(data):
        x |= (c & 0x7F) << shift
        if c & 0x80:
            shift += 7
            if shift >= 35:
                raise ValueError("value over 32 bits")
            continue
        if x > 0xFFFFFFFF:
            raise ValueError("value over 32 bits")
        prev += x
        if prev > 0xFFFFFFFF:
            raise ValueError("sum over 32 bits")
        vals.append(prev)
        x, shift = 0, 0
    if shift:
        raise ValueError("payload ends inside a value")
    return vals


def sancov(cov):
    """tools/syz-execprog/execprog.go:165-168: u64 LE 0xC0BFFFFFFFFFFF64, then
    cover.RestorePC(pc, 0xffffffff) (cover.go:23-25) per PC."""
    import struct

    return struct.pack("<Q", 0xC0BFFFFFFFFFFF64) + b"".join(struct.pack("<Q", (0xFFFFFFFF << 32) + int(pc))
                                                           for pc in cov)


def _csr(lists):
    off = np.zeros(len(lists) + 1, dtype=np.uint64)
    if lists:
        off[1:] = np.cumsum([len(x) for x in lists])
    vals = np.concatenate([_u32(x) for x in lists]) if lists else np.zeros(0, np.uint32)
    return vals.astype(np.uint32), off


def triage_batch(maxset, newset, vals, off):
    vals, off = _u32(vals), _u64(off)
    nrec = off.size - 1
    rec_new = np.zeros(nrec, dtype=np.uint8)
    dv = np.empty(max(vals.size, 1), dtype=np.uint32)
    do = np.empty(nrec + 1, dtype=np.uint64)
    nd = L.orc_triage_batch(maxset.h, newset.h if newset is not None else None, p32(vals), p64(off), nrec, p8(rec_new), p32(dv),
                            p64(do))
    return rec_new, dv[:nd].copy(), do


def triage_flags_only(maxset, newset, vals, off):
    vals, off = _u32(vals), _u64(off)
    nrec = off.size - 1
    rec_new = np.zeros(nrec, dtype=np.uint8)
    L.orc_triage_batch(maxset.h, newset.h if newset is not None else None, p32(vals), p64(off), nrec, p8(rec_new), None, None)
    return rec_new


def triage_procs(maxset, newset, vals, off, prog_rec, nthreads):
    """The fuzzer's concurrent procs (timing only: racy by design, like the
    reference).  Returns (rec_new, threads used)."""
    vals, off, pr = _u32(vals), _u64(off), _u64(prog_rec)
    rec_new = np.zeros(off.size - 1, dtype=np.uint8)
    t = L.orc_triage_procs(maxset.h, newset.h if newset is not None else None, p32(vals), p64(off), p64(pr),
                           pr.size - 1, int(nthreads), p8(rec_new))
    return rec_new, t


def add_inputs(corpus, maxset, vals, off):
    vals, off = _u32(vals), _u64(off)
    L.orc_add_inputs(corpus.h, maxset.h, p32(vals), p64(off), off.size - 1)


def accept_batch(corpus_sig, corpus_cov, sv, so, cv=None, co=None):
    sv, so = _u32(sv), _u64(so)
    n = so.size - 1
    acc = np.zeros(n, dtype=np.uint8)
    if corpus_cov is not None and cv is not None:
        cv, co = _u32(cv), _u64(co)
        L.orc_accept_batch(corpus_sig.h, corpus_cov.h, p32(sv), p64(so), p32(cv), p64(co), n, p8(acc))
    else:
        L.orc_accept_batch(corpus_sig.h, None, p32(sv), p64(so), None, None, n, p8(acc))
    return acc


def merge_poll(mgr_max, av, ao):
    av, ao = _u32(av), _u64(ao)
    npoll = ao.size - 1
    nv = np.empty(max(av.size, 1), dtype=np.uint32)
    no = np.empty(npoll + 1, dtype=np.uint64)
    m = L.orc_merge_poll(mgr_max.h, p32(av), p64(ao), npoll, p32(nv), p64(no))
    return nv[:m].copy(), no


def minimize_order(off):
    off = _u64(off)
    n = off.size - 1
    order = np.empty(max(n, 1), dtype=np.uint32)
    L.orc_minimize_order(p64(off), n, p32(order))
    return order[:n].copy()


def minimize(vals, off, order=None):
    vals, off = _u32(vals), _u64(off)
    n = off.size - 1
    order = minimize_order(off) if order is None else _u32(order)
    out = np.empty(max(n, 1), dtype=np.uint32)
    m = L.orc_minimize_ordered(p32(vals), p64(off), n, p32(order), p32(out))
    return out[:m].copy()


def exec_hash(a):
    return L.orc_exec_hash(int(a))


def exec_signal(pcs, call_off, prog_off):
    p, co, po = _u32(pcs), _u64(call_off), _u64(prog_off)
    ncalls = co.size - 1
    out = np.empty(max(p.size, 1), dtype=np.uint32)
    so = np.empty(ncalls + 1, dtype=np.uint64)
    m = L.orc_exec_signal_batch(p32(p), p64(co), p64(po), po.size - 1, p32(out), p64(so))
    return out[:m].copy(), so


def cover_uncovered(cov, base, sym_start, sym_end, all_pcs):
    c, ss, se, ap = _u32(cov), _u64(sym_start), _u64(sym_end), _u64(all_pcs)
    out = np.empty(max(ap.size, 1), dtype=np.uint64)
    n = L.orc_cover_uncovered(p32(c), c.size, base, p64(ss), p64(se), ss.size, p64(ap), ap.size, p64(out))
    return out[:n].copy()


# ---- the compiled reference executor (oracle/_ref) ------------------------------
_ref = None


def ref_executor():
    """ctypes handle of the reference executor, or None if it was not built."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        R = ctypes.CDLL(REF_SO)
        R.ref_exec_hash.restype = c_uint32
        R.ref_exec_hash.argtypes = [c_uint32]
        R.ref_exec_reset.restype = None
        R.ref_exec_reset.argtypes = []
        R.ref_exec_dedup.restype = c_int
        R.ref_exec_dedup.argtypes = [c_uint32]
        R.ref_exec_call_signal.restype = c_uint32
        R.ref_exec_call_signal.argtypes = [P32, c_uint32, P32]
        _ref = R
    return _ref


def ref_exec_signal(pcs, call_off, prog_off):
    """Per-call signal from the reference executor's own hash()/dedup()."""
    R = ref_executor()
    if R is None:
        raise RuntimeError("oracle/_ref/libref_executor.so not built (needs the reference checkout)")
    p, co, po = _u32(pcs), _u64(call_off), _u64(prog_off)
    out = np.empty(max(p.size, 1), dtype=np.uint32)
    so = np.zeros(co.size, dtype=np.uint64)
    m = 0
    for prog in range(po.size - 1):
        R.ref_exec_reset()  # fresh table per program (fork per program)
        for c in range(int(po[prog]), int(po[prog + 1])):
            so[c] = m
            seg = p[int(co[c]): int(co[c + 1])]
            tmp = np.empty(max(seg.size, 1), dtype=np.uint32)
            k = R.ref_exec_call_signal(p32(np.ascontiguousarray(seg)), seg.size, p32(tmp))
            out[m: m + k] = tmp[:k]
            m += k
    so[-1] = m
    return out[:m].copy(), so
