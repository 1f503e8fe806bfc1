#!/usr/bin/env python3
"""The claim path's global-atomic rate (north_star: "HBM GB/s and atomic
throughput achieved against the MI355X peak are shown in rocprof").

run:      python3 scripts/atomic_rate.py run OUT.json
    One C2 batch (bench.py's recipe) against its 16M-entry maxSignal through
    the claim/resolve path (sg_triage_batch_dev with the ordered diff lists:
    k_claim's read-checked atomicMin into the 2^32-entry first-owner table,
    sg_triage.hip), 3 times after a warm-up, HIP-event kernel times; and the
    C4 Minimize claim (k_min_claim, sg_merge.hip) on bench_rows.py's corpus.
pmc:      rocprofv3 --pmc TCC_ATOMIC TCP_TOTAL_ATOMIC_WITH_RET TCP_TOTAL_ATOMIC_WITHOUT_RET
          -d DIR -o run --output-format csv -- python3 scripts/atomic_rate.py run /dev/null
summary:  python3 scripts/atomic_rate.py summary OUT.json PMC.csv MICRO.txt FINAL.json
    atomics per launch (TCC_ATOMIC summed over the L2 channels, per dispatch)
    over the HIP-event kernel time, against the random-address peak of
    scripts/micro/atomics.hip."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out_path):
    import ctypes

    import torch

    import bench
    from bench import Gen, SignalSet, build_m0, call, triage
    from syzkaller_amd.cover import Context

    cfg = {"programs": 65536, "calls": 16, "pcs_per_call": 1024, "zipf_s": 1.1, "ranks": 1 << 20}
    ctx = Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    g = Gen(cfg)
    warm = g.zipf(ctx, cfg, 2_000_000)
    b = g.zipf(ctx, cfg, 1_002)
    del g
    rec_new = torch.empty(b.nrec, dtype=torch.uint8, device="cuda")
    m0, ms = SignalSet(ctx), SignalSet(ctx)
    build_m0(ctx, m0, warm, cfg["calls"], 16 << 20, rec_new)
    del warm
    cnt = ctypes.c_uint64()
    call("sg_set_count_missing_dev", m0.h, b.vals.data_ptr(), b.nvals, ctypes.byref(cnt))
    dv = torch.empty(b.nvals, dtype=torch.int32, device="cuda")
    do = torch.empty(b.nrec + 1, dtype=torch.int64, device="cuda")
    call("sg_set_copy", ms.h, m0.h)
    triage(ctx, ms, None, b, rec_new, dv, do)  # warm-up (owner table allocated)
    torch.cuda.synchronize()
    ctx.timing(True)
    for _ in range(3):
        call("sg_set_copy", ms.h, m0.h)
        triage(ctx, ms, None, b, rec_new, dv, do)
    torch.cuda.synchronize()
    kt = bench.kernel_table(ctx, ["triage_claim", "triage_resolve", "emit", "scan"], 3)
    ctx.timing(False)
    res = {"c2_claim_path": {"n_in": b.nvals, "n_cand": cnt.value, "n_rec": b.nrec, "kernels": kt,
                             "n_diff": int(do[b.nrec].item())}}
    del dv, do, b
    torch.cuda.empty_cache()
    # C4: the Minimize claim over bench_rows.py's 500k-input corpus recipe
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(4)
    n = 500_000
    lens = np.clip(np.exp(rng.normal(np.log(1000), 1.0, size=n)), 1, 16384).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    vt = torch.empty(int(off[-1]), dtype=torch.int32, device="cuda")
    call("sg_gen_zipf_traces_dev", ctx.h, bench.UNIVERSE_SEED, 8402, 1.1, 1 << 22, 0, 1, 1, vt.numel(), vt.data_ptr())
    vals = vt.cpu().numpy().view(np.uint32)
    del vt
    order = C.minimize_order(off)
    C.minimize_csr(vals, off, order, ctx=ctx)  # warm-up
    ctx.timing(True)
    for _ in range(3):
        C.minimize_csr(vals, off, order, ctx=ctx)
    kt4 = bench.kernel_table(ctx, ["min_claim", "min_owners", "scan", "emit"], 3)
    ctx.timing(False)
    res["c4_minimize"] = {"elements": int(vals.size), "inputs": n, "kernels": kt4}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def summary(times_json, pmc_csv, micro_txt, out_json):
    import csv
    from collections import defaultdict

    t = json.load(open(times_json))
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> sum over dims
    for r in csv.DictReader(open(pmc_csv)):
        name = r["Kernel_Name"]
        key = ("k_claim" if "k_claim<" in name else "k_resolve" if "k_resolve<" in name else
               "k_min_claim" if "k_min_claim" in name else None)
        if key:
            per[(key, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    launches = defaultdict(list)
    for (k, _), cs in per.items():
        launches[k].append(cs)
    peak = {}
    for line in open(micro_txt):
        p = line.split()
        if len(p) == 5 and p[1] == "MiB":
            peak[int(p[0])] = {"no_return": float(p[2]), "returning": float(p[3]), "read_checked": float(p[4])}
    big = peak.get(16384) or (peak[max(peak)] if peak else None)
    out = {"source": {"times": times_json, "pmc": pmc_csv, "micro": micro_txt}, "peak_random_16GiB": big,
           "peak_table": peak, "kernels": {}}
    ktime = {"k_claim": t["c2_claim_path"]["kernels"].get("triage_claim", {}).get("avg_ms"),
             "k_resolve": t["c2_claim_path"]["kernels"].get("triage_resolve", {}).get("avg_ms"),
             "k_min_claim": t["c4_minimize"]["kernels"].get("min_claim", {}).get("avg_ms")}
    for k, ls in launches.items():
        avg = {c: float(np.mean([l[c] for l in ls])) for c in ls[0]}
        ms = ktime.get(k)
        atom = avg.get("TCC_ATOMIC")
        rate = atom / (ms / 1e3) / 1e9 if atom and ms else None
        out["kernels"][k] = {"launches_profiled": len(ls), "counters_per_launch": avg, "avg_ms_events": ms,
                             "atomics_per_s_G": rate,
                             "frac_of_random_peak": (rate / big["no_return"]) if rate and big else None}
    out["c2_claim_path"] = t["c2_claim_path"]
    out["c4_minimize"] = t["c4_minimize"]
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summary(*sys.argv[2:6])
