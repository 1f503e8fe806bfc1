"""Regenerate the golden fixtures under tests/golden/ from the reference.

Run in the build container (where the reference checkout exists):
    python tests/golden/make_golden.py [/root/reference]

1. cover_kats.json: the known-answer tables of pkg/cover/cover_test.go
   (TestCanonicalize :60-66, TestDifference :68-76, TestSymmetricDifference
   :78-85, TestUnion :87-94, TestIntersection :96-102, TestMinimize
   :104-157), extracted from the Go source text as data, with each table's
   `sorted` / `symmetric` flags (runTest, cover_test.go:31-58).
2. exec_signal_golden.npz: synthetic KCOV-like traces and the per-call
   signal the REFERENCE executor produces for them -- its own hash()/dedup()
   (executor/executor.h:497-526) driven by the signal loop of
   handle_completion (:389-401), compiled from the reference sources by
   oracle/Makefile into oracle/_ref/.
The reference itself never travels; only these data files do.
"""
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def _ints(s):
    s = s.strip()
    return [int(x, 0) for x in s.split(",") if x.strip()] if s else []


def parse_cover_kats(ref):
    src = open(os.path.join(ref, "pkg/cover/cover_test.go")).read()
    funcs = re.split(r"\nfunc ", src)
    out = {}
    for body in funcs:
        m = re.match(r"(Test\w+)\(", body)
        if not m:
            continue
        name = m.group(1)
        if name == "TestMinimize":
            cases = []
            for cm in re.finditer(r"\[\]Cover\{(.*?)\n\s*\},\s*\[\]int\{([^}]*)\}", body, re.S):
                covs = [_ints(x) for x in re.findall(r"\{([^{}]*)\}", cm.group(1))]
                cases.append({"inp": covs, "out": _ints(cm.group(2))})
            out[name] = {"cases": cases}
            continue
        rm = re.search(r"runTest\(t,.*?,\s*(true|false),\s*(true|false),\s*\[\]Test\{", body, re.S)
        if not rm:
            continue
        cases = [
            {"v0": _ints(a), "v1": _ints(b), "r": _ints(c)}
            for a, b, c in re.findall(r"\{Cover\{([^}]*)\},\s*Cover\{([^}]*)\},\s*Cover\{([^}]*)\}\}", body)
        ]
        out[name] = {"sorted": rm.group(1) == "true", "symmetric": rm.group(2) == "true", "cases": cases}
    return out


def write_kats(f, kats):
    """One KAT case per line."""
    f.write('{"source": "pkg/cover/cover_test.go", "tests": {\n')
    items = list(kats.items())
    for i, (name, t) in enumerate(items):
        meta = "".join("%s: %s, " % (json.dumps(k), json.dumps(v)) for k, v in t.items() if k != "cases")
        f.write(" %s: {%s\"cases\": [\n" % (json.dumps(name), meta))
        f.write(",\n".join("  " + json.dumps(c) for c in t["cases"]))
        f.write("]}" + ("," if i < len(items) - 1 else "") + "\n")
    f.write("}}\n")


def make_exec_golden():
    from oracle import pyoracle

    pyoracle.build()
    rng = np.random.default_rng(20171012)
    progs = []
    # edge cases first: empty program, empty call, zero PC, repeated PCs,
    # a long call that overflows the 8192-slot table (evictions), many calls.
    progs.append([])
    progs.append([[], [0x81000000]])
    progs.append([[0, 0, 0], [5, 5, 5, 5]])
    progs.append([[0x81000010] * 40 + [0x81000020] * 40])
    progs.append([list(rng.integers(0x81000000, 0x81000000 + 16 * 4096, size=20000, dtype=np.uint64) & ~np.uint64(15))])
    for _ in range(24):
        ncalls = int(rng.integers(1, 10))
        calls = []
        for _ in range(ncalls):
            n = int(rng.integers(0, 1500))
            ranks = np.minimum(rng.zipf(1.1, size=n), 1 << 16) - 1
            calls.append(list(0x81000000 + 16 * ranks))
        progs.append(calls)
    pcs, call_off, prog_off = [], [0], [0]
    for calls in progs:
        for c in calls:
            pcs.extend(int(x) & 0xFFFFFFFF for x in c)
            call_off.append(len(pcs))
        prog_off.append(len(call_off) - 1)
    pcs = np.array(pcs, dtype=np.uint32)
    call_off = np.array(call_off, dtype=np.uint64)
    prog_off = np.array(prog_off, dtype=np.uint64)
    sig, sig_off = pyoracle.ref_exec_signal(pcs, call_off, prog_off)
    hin = np.array([0, 1, 61, 0xFFFFFFFF, 0x81000000, 0xDEADBEEF, 12345678], dtype=np.uint32)
    R = pyoracle.ref_executor()
    hout = np.array([R.ref_exec_hash(int(x)) for x in hin], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "exec_signal_golden.npz"), pcs=pcs, call_off=call_off, prog_off=prog_off,
                        sig=sig, sig_off=sig_off, hash_in=hin, hash_out=hout)
    return pcs.size, sig.size


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    kats = parse_cover_kats(ref)
    with open(os.path.join(HERE, "cover_kats.json"), "w") as f:
        write_kats(f, kats)
    print("cover KAT tables:", {k: len(v["cases"]) for k, v in kats.items()})
    print("executor golden: pcs=%d signal=%d" % make_exec_golden())


if __name__ == "__main__":
    main()
