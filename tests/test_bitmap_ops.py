"""The prefix protocol's bitmap passes (include/syzsig.h): the per-rank
prefix OR (sg_bitmap_prefix_or_rank_dev, quad and word paths) against
sg_bitmap_prefix_or_dev and numpy, and the fused set update
(sg_set_or_new_or_dev) against sg_set_or_new_dev followed by sg_set_or_dev."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("words", [4096 * 5, 1001, 4])
@pytest.mark.parametrize("nparts", [1, 3])
def test_prefix_or_rank(ctx, words, nparts):
    from syzkaller_amd._lib import call

    rng = np.random.default_rng(words + nparts)
    parts = rng.integers(0, 1 << 32, size=nparts * words, dtype=np.uint64).astype(np.uint32)
    parts[rng.random(parts.size) < 0.7] = 0  # mostly empty words, as in a low-novelty batch
    dp = torch.from_numpy(parts.view(np.int32)).cuda()
    p = parts.reshape(nparts, words)
    full_pref = torch.empty(nparts * words, dtype=torch.int32, device="cuda")
    full_tot = torch.empty(words, dtype=torch.int32, device="cuda")
    call("sg_bitmap_prefix_or_dev", ctx.h, dp.data_ptr(), nparts, words, full_pref.data_ptr(), full_tot.data_ptr())
    for rank in range(nparts):
        pref = torch.full((words,), -1, dtype=torch.int32, device="cuda")
        tot = torch.full((words,), -1, dtype=torch.int32, device="cuda")
        call("sg_bitmap_prefix_or_rank_dev", ctx.h, dp.data_ptr(), nparts, words, rank,
             ctypes.c_void_p(pref.data_ptr()), tot.data_ptr())
        torch.cuda.synchronize()
        exp_p = np.bitwise_or.reduce(p[:rank], axis=0) if rank else np.full(words, 0xFFFFFFFF, np.uint32)
        assert np.array_equal(pref.cpu().numpy().view(np.uint32), exp_p)  # rank 0's is left untouched
        assert np.array_equal(tot.cpu().numpy().view(np.uint32), np.bitwise_or.reduce(p, axis=0))
        assert torch.equal(tot, full_tot)
        if rank:
            assert torch.equal(pref, full_pref[rank * words:(rank + 1) * words])


def test_set_or_new_or(ctx):
    """Word-wise over sets wrapping torch tensors: newsig |= t & ~maxsig, then
    maxsig |= t; with newsig NULL only maxsig changes."""
    from syzkaller_amd._lib import call
    from syzkaller_amd.shard import _WrappedSet

    W = 1 << 27
    g = torch.Generator(device="cuda").manual_seed(5)

    def sparse(frac):
        t = torch.randint(-(1 << 31), (1 << 31) - 1, (W,), dtype=torch.int32, device="cuda", generator=g)
        keep = torch.rand(W, device="cuda", generator=g) < frac
        return torch.where(keep, t, torch.zeros_like(t))

    m0, n0, t = sparse(0.3), sparse(0.1), sparse(0.02)
    m, n = m0.clone(), n0.clone()
    ms, ns = _WrappedSet(ctx, m), _WrappedSet(ctx, n)
    call("sg_set_or_new_or_dev", ns.h, ms.h, ctypes.c_void_p(t.data_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(n, n0 | (t & ~m0))
    assert torch.equal(m, m0 | t)
    m2 = m0.clone()
    ms2 = _WrappedSet(ctx, m2)
    call("sg_set_or_new_or_dev", None, ms2.h, ctypes.c_void_p(t.data_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(m2, m0 | t)
    from syzkaller_amd._lib import SyzSigError

    with pytest.raises(SyzSigError):  # words aliasing maxsig
        call("sg_set_or_new_or_dev", ns.h, ms.h, ctypes.c_void_p(m.data_ptr()))
    with pytest.raises(SyzSigError):  # newsig == maxsig
        call("sg_set_or_new_or_dev", ms.h, ms.h, ctypes.c_void_p(t.data_ptr()))
    for s_ in (ms, ns, ms2):
        s_.close()
