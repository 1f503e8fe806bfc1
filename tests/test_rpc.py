"""RPC payload forms (pkg/rpctype/rpctype.go:8-63) and
the sancov dump (tools/syz-execprog/execprog.go:159-177): the oracle against
Go's encoding rules (CPU), the product's encoders / decoders against the
oracle bit-exactly and round-tripping the []uint32 form (GPU)."""
import numpy as np
import pytest

from oracle import pyoracle as O


def test_uvarint_matches_go_encoding():
    # binary.PutUvarint reference points (LEB128)
    assert O.put_uvarint(0) == b"\x00"
    assert O.put_uvarint(127) == b"\x7f"
    assert O.put_uvarint(128) == b"\x80\x01"
    assert O.put_uvarint(300) == b"\xac\x02"
    assert O.put_uvarint(0xFFFFFFFF) == b"\xff\xff\xff\xff\x0f"
    rng = np.random.default_rng(41)
    for _ in range(50):
        v = np.unique(rng.integers(0, 1 << 32, size=int(rng.integers(0, 500)), dtype=np.uint64)).astype(np.uint32)
        assert O.delta_decode(O.delta_encode(v)) == [int(x) for x in v]
    for bad in (b"\x80", b"\xff\xff\xff\xff\x1f", b"\xff\xff\xff\xff\x0f\x01"):
        with pytest.raises(ValueError):
            O.delta_decode(bad)


def test_delta_encode_batch_matches_per_list_oracle():
    """The vectorised batch encoder (the f4 row's full-payload check) gives the
    per-list oracle's bytes: empty lists, value 0 and 0xFFFFFFFF, repeats
    (delta 0), deltas at every varint length boundary."""
    rng = np.random.default_rng(43)
    lists = [np.zeros(0, np.uint32), np.array([0], np.uint32), np.array([0xFFFFFFFF], np.uint32),
             np.array([5, 5, 5], np.uint32), np.cumsum([127, 1, 16383, 1, 2097151, 1, 268435455, 1]).astype(np.uint32)]
    for _ in range(300):
        v = np.sort(rng.integers(0, 1 << 32, size=int(rng.integers(0, 60)), dtype=np.uint64)).astype(np.uint32)
        lists.append(v if rng.random() < 0.5 else np.unique(v))
    vals = np.concatenate(lists).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum([x.size for x in lists])]).astype(np.uint64)
    b, bo = O.delta_encode_batch(vals, off)
    for k, x in enumerate(lists):
        assert b[int(bo[k]):int(bo[k + 1])].tobytes() == O.delta_encode(x), k


def test_sancov_layout():
    b = O.sancov([0x81000010, 5])
    assert b[:8] == bytes.fromhex("64ffffffffffbfc0")
    assert b[8:16] == (0xFFFFFFFF81000010).to_bytes(8, "little")
    assert len(b) == 24


def _lists(rng, n):
    out = []
    for k in range(n):
        m = int(rng.integers(0, 3000)) if k % 9 else 0
        if k % 3 == 0:   # edge signal: spread over 32 bits
            v = rng.integers(0, 1 << 32, size=m, dtype=np.uint64)
        else:            # cover: clustered kernel-text PCs, duplicates (multisets sort fine)
            v = 0x81000000 + 16 * rng.integers(0, 1 << 16, size=m)
        v = np.sort(v).astype(np.uint32)
        if k == 5 and m:
            v[-1] = 0xFFFFFFFF
        out.append(v)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("blocks", ["0", "1"])  # the wave-per-list codec / the per-block and per-element forms
def test_delta_batch_vs_oracle(ctx, ctx_option, blocks):
    from syzkaller_amd import cover as C

    ctx_option(ctx, "rpc_decode_blocks", int(blocks))
    ctx_option(ctx, "rpc_encode_elems", int(blocks))

    rng = np.random.default_rng(42)
    lists = _lists(rng, 200)
    vals, off = C.to_csr(lists)
    data, doff = C.delta_encode(vals, off, ctx=ctx)
    for k, v in enumerate(lists):
        assert data[int(doff[k]):int(doff[k + 1])].tobytes() == O.delta_encode(v), k
    gv, go = C.delta_decode(data, doff, ctx=ctx)
    assert np.array_equal(go, off) and np.array_equal(gv, vals)
    # not sorted -> rejected
    from syzkaller_amd._lib import SyzSigError
    with pytest.raises(SyzSigError):
        C.delta_encode(np.array([5, 3], np.uint32), np.array([0, 2], np.uint64), ctx=ctx)
    # a descent exactly across the encoder's 64-value step, in the 2nd list
    u = np.arange(300, dtype=np.uint32)
    u[64] = 62
    with pytest.raises(SyzSigError):
        C.delta_encode(np.concatenate([u[:10], u]), np.array([0, 10, 310], np.uint64), ctx=ctx)
    # ... but a list may start below the previous one's end
    w = np.concatenate([np.arange(100, 200, dtype=np.uint32), np.arange(0, 64, dtype=np.uint32)])
    wd, wo = C.delta_encode(w, np.array([0, 100, 164], np.uint64), ctx=ctx)
    assert wd.tobytes() == O.delta_encode(w[:100]) + O.delta_encode(w[100:])
    # malformed payloads -> rejected
    for bad in (b"\x05\x80", b"\xff\xff\xff\xff\x1f", b"\xff\xff\xff\xff\x0f\x01", b"\xff\xff\xff\xff\xff\x01"):
        with pytest.raises(SyzSigError):
            C.delta_decode(bad, np.array([0, len(bad)], np.uint64), ctx=ctx)
    # a list may not end inside a value even when the next one would complete it
    with pytest.raises(SyzSigError):
        C.delta_decode(b"\x81\x01", np.array([0, 1, 2], np.uint64), ctx=ctx)


@pytest.mark.gpu
def test_delta_codec_list_edges(ctx, ctx_option):
    """The per-list codec at every 16-byte / 4-value alignment: lists of 0-9
    and 255-257 values (steps of 256 values and 1 KiB, loads aligned down to
    the list's first value / byte), values 0 and 0xFFFFFFFF, long zero runs
    (1-byte varints) and maximal deltas (5-byte varints), 300 lists so the
    default routing takes the per-list kernels."""
    from syzkaller_amd import cover as C

    assert ctx.get_option("rpc_decode_blocks") == -1 and ctx.get_option("rpc_encode_elems") == -1
    rng = np.random.default_rng(48)
    lists = []
    for k in range(300):
        m = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 255, 256, 257][k % 13]
        kind = k % 3
        if kind == 0:
            v = np.zeros(m, np.uint32)
        elif kind == 1:
            v = np.sort(rng.integers(0, 1 << 32, size=m, dtype=np.uint64)).astype(np.uint32)
            if m:
                v[0], v[-1] = 0, 0xFFFFFFFF
        else:
            v = np.sort(rng.integers(0, 300, size=m)).astype(np.uint32)
        lists.append(np.sort(v))
    vals, off = C.to_csr(lists)
    data, doff = C.delta_encode(vals, off, ctx=ctx)
    exp = b"".join(O.delta_encode(v) for v in lists)
    assert data.tobytes() == exp
    gv, go = C.delta_decode(data, doff, ctx=ctx)
    assert np.array_equal(go, off) and np.array_equal(gv, vals)


@pytest.mark.gpu
def test_set_payload_round_trip(ctx):
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(43)
    m = np.unique(rng.integers(0, 1 << 32, size=300000, dtype=np.uint64)).astype(np.uint32)
    m = np.concatenate([m, np.array([0, 0xFFFFFFFF], np.uint32)])
    s = C.SignalSet(ctx)
    C.SignalAdd(s, m)
    payload = C.set_encode(s)
    exp = np.unique(m)
    assert payload == O.delta_encode(exp)
    assert len(payload) < 4 * exp.size  # smaller than the []uint32 form
    t = C.SignalSet(ctx)
    C.SignalAdd(t, np.array([7, 8, 9], np.uint32))
    assert C.set_decode_add(t, payload) == exp.size  # SignalAdd of the payload
    assert np.array_equal(t.export(), np.union1d(exp, [7, 8, 9]).astype(np.uint32))
    e = C.SignalSet(ctx)
    assert C.set_encode(e) == b""
    assert C.set_decode_add(e, b"") == 0 and len(e) == 0
    for x in (s, t, e):
        x.close()


@pytest.mark.gpu
def test_sancov_batch_vs_oracle(ctx):
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(44)
    covs = [(0x81000000 + 16 * rng.integers(0, 1 << 20, size=int(rng.integers(0, 500)))).astype(np.uint32)
            for _ in range(64)]
    covs[3] = np.zeros(0, np.uint32)
    vals, off = C.to_csr(covs)
    files = C.sancov(vals, off, ctx=ctx)
    assert len(files) == len(covs)
    for k, c in enumerate(covs):
        assert files[k] == O.sancov(c), k


@pytest.mark.gpu
@pytest.mark.parametrize("blocks", ["0", "1"])
def test_delta_decode_corrupted_payloads_vs_oracle(ctx, ctx_option, blocks):
    """Decode accepts / rejects exactly what binary.Uvarint + a running sum do
    (oracle), on payloads with flipped high bits and cut ends, including runs
    that cross the decoder's 32-byte blocks, its 1 KiB wave steps and list
    boundaries."""
    from syzkaller_amd import cover as C
    from syzkaller_amd._lib import SyzSigError

    ctx_option(ctx, "rpc_decode_blocks", int(blocks))
    rng = np.random.default_rng(7)
    for t in range(160):
        parts = []
        for _ in range(int(rng.integers(1, 4))):
            m = int(rng.integers(0, 60 if t < 120 else 1500))
            v = np.sort(rng.integers(0, 1 << 32, size=m, dtype=np.uint64)).astype(np.uint32)
            parts.append(bytearray(O.delta_encode(v)))
        for p in parts:
            if p and rng.random() < 0.7:
                for _ in range(int(rng.integers(1, 4))):
                    p[int(rng.integers(0, len(p)))] ^= 0x80
            if p and rng.random() < 0.2:
                del p[int(rng.integers(0, len(p))):]
        expect = []
        try:
            for p in parts:
                expect.append(O.delta_decode(bytes(p)))
        except ValueError:
            expect = None
        data = b"".join(bytes(p) for p in parts)
        doff = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.uint64)
        if expect is None:
            with pytest.raises(SyzSigError):
                C.delta_decode(data, doff, ctx=ctx)
            continue
        gv, go = C.delta_decode(data, doff, ctx=ctx)
        assert [gv[int(go[k]):int(go[k + 1])].tolist() for k in range(len(parts))] == expect, t


@pytest.mark.gpu
@pytest.mark.parametrize("blocks", ["0", "1"])
def test_delta_decode_sum_past_32_bits(ctx, ctx_option, blocks):
    """A running sum that passes 2^32 - 1 at a chosen value, deep in a long
    list (across the decoder's lanes, rows and steps): rejected exactly when
    binary.Uvarint + the sum would overflow the uint32 (oracle), accepted when
    it ends at 0xFFFFFFFF."""
    from syzkaller_amd import cover as C
    from syzkaller_amd._lib import SyzSigError

    ctx_option(ctx, "rpc_decode_blocks", int(blocks))
    step = (1 << 24) + 1
    for m, last in ((300, None), (255, None), (256, None), (257, None), (1000, None), (255, 0xFFFFFFFF)):
        d = [step] * m
        if last is not None:
            d[-1] = last - step * (m - 1)
        payload = b"".join(O.put_uvarint(x) for x in d)
        lead = O.delta_encode(np.arange(0, 700, 3, dtype=np.uint32))
        data = lead + payload
        doff = np.array([0, len(lead), len(data)], np.uint64)
        try:
            expect = [O.delta_decode(lead), O.delta_decode(payload)]
        except ValueError:
            expect = None
        if expect is None:
            with pytest.raises(SyzSigError):
                C.delta_decode(data, doff, ctx=ctx)
            continue
        gv, go = C.delta_decode(data, doff, ctx=ctx)
        assert [gv[int(go[k]):int(go[k + 1])].tolist() for k in range(2)] == expect, m
