"""oracle/ipc_oracle.py -- TEST INFRASTRUCTURE ONLY (the checker of
sg_ipc_parse; the product never imports it).

Pure-Python restatement of the executor output reader
`pkg/ipc/ipc_linux.go:168-307` (readOutCoverage), one Go statement per step,
and of the writer side `executor/executor.h:369-427` + `:621-648`
(kcov_comparison_t::write) used to build test inputs.

Parity unpinned by reference fixtures: the reference holds no golden output
buffer or test of readOutCoverage (pkg/ipc/ipc_test.go runs a live
executor), so this restatement follows the cited lines only.
"""

OK, NO_NCMD, SHORT_HEADER, BAD_INDEX, BAD_CALLNUM, DOUBLE = 0, 1, 2, 3, 4, 5
SIGNAL_SIZE, COVER_SIZE, COMPS_SHORT, COMPS_TYPE = 6, 7, 8, 9

COMP_SIZE_MASK, COMP_SIZE8, COMP_CONST_MASK = 6, 6, 1  # ipc_linux.go:41-43


def read_out_coverage(out, ncalls, call_nums=None):
    """ipc_linux.go:168-307 over one program's output words.  Returns
    (status, info) with info[i] = dict(errno, fault, signal, cover); signal /
    cover are None while Go's slices are nil."""
    out = [int(x) & 0xFFFFFFFF for x in out]
    pos = 0

    def read():  # readOut (:170-177)
        nonlocal pos
        if pos >= len(out):
            return None
        v = out[pos]
        pos += 1
        return v

    info = [dict(errno=-1, fault=0, signal=None, cover=None) for _ in range(ncalls)]  # :201-205
    ncmd = read()
    if ncmd is None:  # :197-200
        return NO_NCMD, info
    for _ in range(ncmd):
        hdr = [read() for _ in range(7)]  # :216 (readOut short-circuits; no side effects)
        if any(v is None for v in hdr):
            return SHORT_HEADER, info
        idx, num, errno, fi, nsig, ncov, ncomps = hdr
        if idx >= ncalls:  # :220
            return BAD_INDEX, info
        if call_nums is not None and int(call_nums[idx]) != num:  # :225-226
            return BAD_CALLNUM, info
        if info[idx]["signal"] is not None:  # :231
            return DOUBLE, info
        info[idx]["errno"] = errno  # :236 (int(uint32))
        info[idx]["fault"] = 1 if fi != 0 else 0
        if nsig > len(out) - pos:  # :238
            return SIGNAL_SIZE, info
        info[idx]["signal"] = out[pos:pos + nsig]
        pos += nsig
        if ncov > len(out) - pos:  # :247
            return COVER_SIZE, info
        info[idx]["cover"] = out[pos:pos + ncov]
        pos += ncov
        for _ in range(ncomps):  # :257-303, walked without building the CompMap
            typ = read()
            if typ is None:
                return COMPS_SHORT, info
            if typ > COMP_CONST_MASK | COMP_SIZE_MASK:  # :266
                return COMPS_TYPE, info
            k = 2 if (typ & COMP_SIZE_MASK) == COMP_SIZE8 else 4  # the reader's widths (:272-287)
            for _ in range(k):
                if read() is None:
                    return COMPS_SHORT, info
    return OK, info


def write_call(call_index, call_num, errno, fault, signal, cover=(), comps=(), widths="writer"):
    """executor.h:369-427 for one completed call; comps = [(type, arg1, arg2)]
    written as kcov_comparison_t::write does (executor.h:621-648: 4 operand
    words for size-8 comparisons, 2 otherwise).  The reader takes the opposite
    widths (ipc_linux.go:272-287); widths="reader" lays them out the reader's
    way, so that test regions with comparisons parse through."""
    w = [call_index, call_num, errno & 0xFFFFFFFF, fault, len(signal), len(cover), len(comps)]
    w += [int(s) & 0xFFFFFFFF for s in signal]
    w += [int(c) & 0xFFFFFFFF for c in cover]
    for typ, a1, a2 in comps:
        w.append(typ)
        if ((typ & COMP_SIZE_MASK) != COMP_SIZE8) == (widths == "writer"):
            w += [a1 & 0xFFFFFFFF, a2 & 0xFFFFFFFF]
        else:
            w += [a1 & 0xFFFFFFFF, (a1 >> 32) & 0xFFFFFFFF, a2 & 0xFFFFFFFF, (a2 >> 32) & 0xFFFFFFFF]
    return w


def parse_batch(out, out_off, call_off, call_nums=None):
    """The batch contract of sg_ipc_parse, one read_out_coverage per program:
    (errno[], fault[], status[], sig_lists[], cov_lists[]) in record order.
    A program whose read failed keeps its records' errno / fault (the reader's
    partial state) but contributes empty signal / cover lists: execute1
    retries or panics on the error and never returns that info to the triage
    loop (syz-fuzzer/fuzzer.go:752-768)."""
    errs, faults, status, sigs, covs = [], [], [], [], []
    for p in range(len(out_off) - 1):
        r0, r1 = int(call_off[p]), int(call_off[p + 1])
        nums = None if call_nums is None else list(call_nums[r0:r1])
        st, info = read_out_coverage(out[int(out_off[p]):int(out_off[p + 1])], r1 - r0, nums)
        status.append(st)
        for i in info:
            errs.append(i["errno"])
            faults.append(i["fault"])
            sigs.append((i["signal"] or []) if st == OK else [])
            covs.append((i["cover"] or []) if st == OK else [])
    return errs, faults, status, sigs, covs
