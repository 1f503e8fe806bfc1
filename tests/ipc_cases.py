"""Seeded executor output batches for the ipc ingest tests: regions written as
executor/executor.h:369-427 writes them (oracle/ipc_oracle.py write_call),
with every readOutCoverage error path of pkg/ipc/ipc_linux.go:168-307 planted
in some programs."""
import numpy as np

from oracle import ipc_oracle as I

FAULTS = ["ok", "writer_widths", "empty", "short_header", "bad_index", "bad_callnum", "double", "signal_size", "cover_size",
          "comps_short", "comps_type", "trailing", "unexecuted"]


def program(rng, ncalls, nums, kind, maxsig=300, widths="reader"):
    """One program's output region and the kind of damage planted in it."""
    if kind == "writer_widths":  # the executor's own comparison layout (misread by the reader)
        kind, widths = "ok", "writer"
    order = list(rng.permutation(ncalls))  # calls complete in any order
    if kind == "unexecuted" and ncalls:
        order = order[: max(0, ncalls - 2)]
    words = []
    for ci in order:
        nsig = int(rng.integers(0, maxsig))
        sig = rng.integers(0, 1 << 32, size=nsig, dtype=np.uint64)
        cov = rng.integers(0x81000000, 0x82000000, size=int(rng.integers(0, 50)), dtype=np.uint64)
        comps = [(int(rng.integers(0, 8)), int(rng.integers(0, 1 << 63)), int(rng.integers(0, 1 << 63)))
                 for _ in range(int(rng.integers(0, 3)))]
        errno = int(rng.choice([0, 0, 0, 14, 22, 0xFFFFFFFF]))
        words += I.write_call(int(ci), int(nums[ci]), errno, int(rng.integers(0, 2)), sig, cov, comps, widths)
    ncmd = len(order)
    if kind == "empty":
        return []
    if kind == "double" and ncalls:
        words += I.write_call(int(order[0]) if order else 0, int(nums[order[0]]) if order else 0, 0, 0, [1, 2])
        ncmd += 1
    elif kind == "bad_index":
        words += I.write_call(ncalls + int(rng.integers(0, 3)), 0, 0, 0, [5])
        ncmd += 1
    elif kind == "bad_callnum" and ncalls:
        words = I.write_call(0, int(nums[0]) + 1, 0, 0, [7, 8]) + words
        ncmd += 1
    elif kind == "comps_type":
        words += [ncalls, 0, 0, 0, 0, 0, 1, 8 + int(rng.integers(0, 100))]
        ncmd += 1
    elif kind == "trailing":
        words += [int(x) for x in rng.integers(0, 1 << 32, size=int(rng.integers(1, 40)), dtype=np.uint64)]
    words = [ncmd] + words
    if kind == "short_header":
        words = words + [0, 0, 0]
        words[0] += 1
    elif kind in ("signal_size", "cover_size", "comps_short") and len(order):
        # the last record claims more words than the region holds
        w = I.write_call(0 if kind != "signal_size" else ncalls + 0, 0, 0, 0, [])
        w[0] = int(order[-1])
        w[1] = int(nums[order[-1]])
        if kind == "signal_size":
            w[4] = 1000
        elif kind == "cover_size":
            w[5] = 1000
        else:
            w[6] = 3
            w += [6, 1]
        # replace the last call's record by the damaged one: rebuild without it
        words = [ncmd] + _without_last(words[1:], len(order)) + w
    return words


def _without_last(words, n):
    """Drop the last of n records from a well-formed record sequence."""
    pos, starts = 0, []
    for _ in range(n):
        starts.append(pos)
        nsig, ncov, ncomps = words[pos + 4], words[pos + 5], words[pos + 6]
        pos += 7 + nsig + ncov
        for _ in range(ncomps):
            t = words[pos]
            pos += 1 + (2 if (t & 6) == 6 else 4)
    return words[: starts[-1]] if starts else words


def batch(seed, nprog=200, maxcalls=20, kinds=None, maxsig=300):
    rng = np.random.default_rng(seed)
    regions, ncalls, nums = [], [], []
    for _ in range(nprog):
        n = int(rng.integers(0, maxcalls + 1))
        cn = rng.integers(0, 4000, size=n).astype(np.uint32)
        kind = kinds[len(regions) % len(kinds)] if kinds else str(rng.choice(FAULTS, p=_weights()))
        regions.append(program(rng, n, cn, kind, maxsig))
        ncalls.append(n)
        nums.append(cn)
    out_off = np.concatenate([[0], np.cumsum([len(r) for r in regions])]).astype(np.uint64)
    call_off = np.concatenate([[0], np.cumsum(ncalls)]).astype(np.uint64)
    out = np.array([w for r in regions for w in r], dtype=np.uint64).astype(np.uint32)
    call_nums = np.concatenate(nums + [np.zeros(0, np.uint32)]).astype(np.uint32)
    return out, out_off, call_off, call_nums


def _weights():
    w = np.ones(len(FAULTS))
    w[0] = 10.0
    return w / w.sum()
