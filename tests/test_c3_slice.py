"""C3 parity at a per-rank slice's full size (BASELINE.json configs[2]: a
1Mi-program batch over 8 GPUs = 128Ki programs x 16 calls x 1024 PCs per
rank, ~1.76G signal entries).

The batch is the fuzzer's steady state (a population re-executed with flaky
coverage, against maxSignal = the population's signal), split into rank 0's
slice (16Ki programs) and rank 1's (the full 128Ki-program per-rank slice).
Both multi-GPU protocols (syzkaller_amd/shard.py) are checked on one GPU
against the oracle's ONE sequential loop (syz-fuzzer/fuzzer.go:645-693) over
rank 0's records then rank 1's:

  * PrefixTriage, run as rank 1 of 2 (gather mode, the G = 2 form): rank 0's
    bitmap C_0 is computed here and handed in by a stand-in for the
    all-gather, so start() / finish() -- sg_prefix_begin_dev over the whole
    slice (two record slices of <= 2^30 entries kept in a slot),
    sg_bitmap_prefix_or_dev, sg_prefix_end_dev against M0 | P_1 with a
    non-empty prefix, the set updates -- run at full size; then again with
    the sparse exchange (rank 0's candidate list handed in: the pairs form,
    sg_prefix_cands_dev, P_1 set from the list, sg_set_add_new_dev);
  * the pair protocol's stages (sg_shard_candidates_dev over each slice,
    sg_shard_owners_dev per shard over the pairs routed to it,
    sg_shard_flags_dev), the routing done here.
Bit-exact: rank 1's flags, the batch's flags, maxSignal and newSignal."""
import numpy as np
import pytest
import torch

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

UNIVERSE_SEED = 0x5A17C0DE
POP_SEED = 0x9091A7E5
CALLS, PCS = 16, 1024


def _signal(call, ctx, trace, nprog):
    ncalls, npcs = nprog * CALLS, nprog * CALLS * PCS
    call_off = torch.arange(0, npcs + 1, PCS, dtype=torch.int64, device="cuda")
    prog_off = torch.arange(0, ncalls + 1, CALLS, dtype=torch.int64, device="cuda")
    sig = torch.empty(npcs, dtype=torch.int32, device="cuda")
    off = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_dev", ctx.h, trace.data_ptr(), call_off.data_ptr(), prog_off.data_ptr(), nprog, ncalls, npcs,
         sig.data_ptr(), off.data_ptr())
    torch.cuda.synchronize()
    n = int(off[-1].item())
    return sig[:n].clone(), off


class _RankOneOfTwo:
    """Comm of rank 1 in a 2-rank group whose collectives return rank 0's part
    beside this rank's: gather mode's all-gather of the C bitmaps (C_0), the
    all-gather of the (candidates, entries) counts, and the sparse exchange's
    all-gather of the candidate lists (cands0: rank 0's, sorted; None: rank 0
    reports as many candidates as entries, which keeps the exchange dense)."""

    world, rank, host, local = 2, 1, False, False

    def __init__(self, c0, nv0, cands0=None):
        self.c0, self.nv0, self.cands0 = c0, nv0, cands0

    def start_all_gather_equal(self, out, t):
        from syzkaller_amd.shard import _Done

        w = t.numel()
        out[:w].copy_(self.c0)
        out[w:2 * w].copy_(t)
        return _Done()

    def all_gather_equal(self, out, t):
        w = t.numel()
        if t.dtype == torch.int64:  # the counts
            n0 = self.nv0 if self.cands0 is None else self.cands0.numel()
            out[:2].copy_(torch.tensor([n0, self.nv0], dtype=torch.int64, device=out.device))
        else:  # a candidate list, padded to the longest
            out[:w].zero_()
            out[: self.cands0.numel()].copy_(self.cands0)
        out[w:2 * w].copy_(t)
        return out


@pytest.mark.timeout(900)
def test_c3_rank_slice_prefix_and_pairs_vs_oracle(ctx):
    from syzkaller_amd._lib import call
    from syzkaller_amd.shard import HipStages, PrefixTriage

    npop, nprog0, nprog1 = 2048, 16384, 131072
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    st = HipStages(ctx)
    W = st.words
    trace = torch.empty(nprog1 * CALLS * PCS, dtype=torch.int32, device="cuda")
    # M0 = the population's signal
    call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, 1.1, 1 << 20, 0, npop, CALLS, PCS, trace.data_ptr())
    msig, _ = _signal(call, ctx, trace, npop)
    m0 = np.unique(msig.cpu().numpy().view(np.uint32))
    del msig
    # the batch: rank 0's slice = programs [0, nprog0), rank 1's = the next nprog1
    slices = []
    for base, n in ((0, nprog0), (nprog0, nprog1)):
        call("sg_gen_population_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, npop, 7_003, 2e-4, 1.1, 1 << 20, base, n,
             CALLS, PCS, trace.data_ptr())
        slices.append(_signal(call, ctx, trace, n))
    del trace
    (sig0, off0), (sig1, off1) = slices
    nrec0, nrec1 = off0.numel() - 1, off1.numel() - 1
    nv0, nv1 = sig0.numel(), sig1.numel()
    assert nv1 > 1_700_000_000  # the C3 per-rank slice
    m0_dev = torch.from_numpy(m0.view(np.int32)).cuda()

    # the oracle: one sequential loop over rank 0's records, then rank 1's
    om, on = O.OSet(m0), O.OSet()
    ef0 = O.triage_flags_only(om, on, sig0.cpu().numpy().view(np.uint32), off0.cpu().numpy().view(np.uint64))
    ef1 = O.triage_flags_only(om, on, sig1.cpu().numpy().view(np.uint32), off1.cpu().numpy().view(np.uint64))
    assert 0.05 < float(ef1.mean()) < 0.95  # mixed flags: the attribution is really tested
    em, en = om.export(), on.export()
    del om, on

    # --- PrefixTriage as rank 1 of 2 ---------------------------------------
    # C_0 = rank 0's signal not in M0 (its sg_prefix_begin_dev marks)
    all0, m0w = torch.zeros(W, dtype=torch.int32, device="cuda"), torch.zeros(W, dtype=torch.int32, device="cuda")
    s_all0, s_m0 = st.wrap(all0), st.wrap(m0w)
    st.add(s_all0, sig0, nv0)
    st.add(s_m0, m0_dev, m0.size)
    c0 = all0 & ~m0w
    assert int(torch.count_nonzero(c0)) > 0  # a non-empty prefix
    # rank 0's candidate list (its signal not in M0, once each) for the sparse exchange
    sv = sig0.to(torch.int64) & 0xFFFFFFFF
    pos = ((sv & 0x00FFFF00) << 8) | ((sv >> 16) & 0xFF00) | (sv & 0xFF)  # sgd::set_pos
    inm0 = (m0w.to(torch.int64)[pos >> 5] >> (sv & 31)) & 1
    cands0 = torch.unique(sv[inm0 == 0]).to(torch.int32)
    del sv, pos, inm0
    assert 0 < cands0.numel() < nv0 // 20  # the steady state's few candidates
    for exchange in ("dense", "sparse"):  # bitmaps (C_0 gathered), then candidate lists
        ms, ns = st.new_set(), st.new_set()
        st.add(ms, m0_dev, m0.size)
        comm = _RankOneOfTwo(c0, nv0, cands0 if exchange == "sparse" else None)
        tri = PrefixTriage(st, comm, gather=True, exchange=exchange)
        rec_new = torch.zeros(nrec1, dtype=torch.uint8, device="cuda")
        assert tri.step(ms, ns, sig1, off1, nv1, nrec1, nrec0, rec_new, nrec_total=nrec0 + nrec1) == nrec0 + nrec1
        torch.cuda.synchronize()
        assert tri.last["exchange"] == exchange
        assert np.array_equal(rec_new.cpu().numpy(), ef1), exchange
        assert np.array_equal(ms.export(), em), exchange
        assert np.array_equal(ns.export(), en), exchange
        del tri, rec_new, ms, ns
    del c0, all0, m0w, s_all0, s_m0, cands0
    torch.cuda.empty_cache()

    # --- the pair protocol's stages over the two slices, G = 2 --------------
    snap = st.new_set()
    st.add(snap, m0_dev, m0.size)
    ntot = nrec0 + nrec1
    routed = [[], []]
    for (sig, off, nv, nrec), base in (((sig0, off0, nv0, nrec0), 0), ((sig1, off1, nv1, nrec1), nrec0)):
        pairs = torch.empty(2 * nv, dtype=torch.int32, device="cuda")
        so = st.candidates(snap, sig, off, nv, nrec, base, 2, pairs)
        for k in range(2):
            routed[k].append(pairs[2 * so[k]: 2 * so[k + 1]].clone())
        del pairs
    nwords = (ntot + 31) // 32
    bits = torch.zeros(2 * nwords, dtype=torch.int32, device="cuda")
    new = []
    for k in range(2):
        recv = torch.cat(routed[k])
        npairs = recv.numel() // 2
        nv_k = torch.empty(max(npairs, 1), dtype=torch.int32, device="cuda")
        nnew = st.owners(recv, npairs, ntot, bits[k * nwords:(k + 1) * nwords], nv_k)
        new.append(nv_k[:nnew].cpu().numpy().view(np.uint32))
    flags = torch.zeros(ntot, dtype=torch.uint8, device="cuda")
    st.flags(bits, 2, nwords, 0, ntot, flags)
    torch.cuda.synchronize()
    assert np.array_equal(flags.cpu().numpy(), np.concatenate([ef0, ef1]))
    assert np.array_equal(np.sort(np.concatenate(new)), en)  # each new signal once, from its one shard
    call("sg_ctx_reset_stream", ctx.h)
