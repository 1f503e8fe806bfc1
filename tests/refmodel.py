"""Tiny pure-Python restatements used to cross-check the C oracle itself on
small cases (test infrastructure; not the product)."""
from collections import Counter

SENT = 0xFFFFFFFF


def foreach_counts(op, a, b):
    """pkg/cover/cover.go:81-102 by value counts (SURVEY.md §0 finding 3)."""
    ca, cb = Counter(a), Counter(b)
    out = []
    for v in sorted(set(ca) | set(cb)):
        if v == SENT:
            continue
        x, y = ca[v], cb[v]
        k = {0: max(x - y, 0), 1: abs(x - y), 2: max(x, y), 3: min(x, y)}[op]
        out.extend([v] * k)
    return out


def foreach_loop(op, a, b):
    """pkg/cover/cover.go:81-102 line by line."""
    res = []
    i0 = i1 = 0
    while i0 < len(a) or i1 < len(b):
        v0 = a[i0] if i0 < len(a) else SENT
        v1 = b[i1] if i1 < len(b) else SENT
        if v0 <= v1:
            i0 += 1
        if v1 <= v0:
            i1 += 1
        if op == 0:
            v = v0 if v0 < v1 else SENT
        elif op == 1:
            v = v0 if v0 < v1 else (v1 if v1 < v0 else SENT)
        elif op == 2:
            v = v0 if v0 <= v1 else v1
        else:
            v = v0 if v0 == v1 else SENT
        if v != SENT:
            res.append(v)
    return res


def canonicalize(v):
    """pkg/cover/cover.go:28-40."""
    s = sorted(v)
    out, last = [], SENT
    for pc in s:
        if pc != last:
            last = pc
            out.append(pc)
    return out


def triage(maxset, newset, records):
    """syz-fuzzer/fuzzer.go:665-691 with Python sets."""
    flags, diffs = [], []
    for sig in records:
        if not any(s not in maxset for s in sig):
            flags.append(0)
            diffs.append([])
            continue
        diff = [s for s in sig if s not in maxset]
        maxset.update(diff)
        newset.update(diff)
        flags.append(1)
        diffs.append(diff)
    return flags, diffs


def minimize(corpus, order):
    """pkg/cover/cover.go:129-145 over a given order."""
    covered, out = set(), []
    for idx in order:
        hit = False
        for pc in corpus[idx]:
            if not hit and pc not in covered:
                hit = True
                out.append(idx)
            if hit:
                covered.add(pc)
    return out
