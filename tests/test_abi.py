"""The C-ABI library builds, loads and exports exactly what include/syzsig.h
declares; without a GPU every computing entry point fails loudly (no CPU
fallback).  CPU only: no kernel is launched here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "syzsig.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ["sg_triage_batch", "sg_triage_batch_dev", "sg_set_new", "sg_set_diff", "sg_set_add",
                 "sg_canonicalize", "sg_merge", "sg_minimize", "sg_accept_batch", "sg_merge_poll",
                 "sg_exec_signal", "sg_cover_uncovered"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from syzkaller_amd import _lib

    so = _lib.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (sg_[a-z0-9_]+)$", out, flags=re.M))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    # and the ctypes binding covers the whole header, one to one
    assert sorted(_lib.SIGNATURES) == declared()
    lib = ctypes.CDLL(so)
    for n in declared():
        getattr(lib, n)


def test_library_is_gfx950_code_object():
    from syzkaller_amd import _lib

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_no_gpu_fails_loudly():
    from syzkaller_amd._lib import SG_ENODEV, SyzSigError
    from syzkaller_amd.cover import Context

    with pytest.raises(SyzSigError) as e:
        Context(0)
    assert e.value.rc == SG_ENODEV


def test_version_string():
    from syzkaller_amd._lib import lib

    assert b"gfx950" in lib.sg_version()


def test_minimize_order_matches_oracle_go_sort():
    # host-side part of sg_minimize: Go's sort.Sort order restated in the product
    from oracle import pyoracle as O
    from syzkaller_amd.cover import minimize_order

    rng = np.random.default_rng(11)
    for n in [0, 1, 2, 5, 6, 7, 12, 13, 40, 41, 100, 1000, 20000]:
        for lenhi in [2, 5, 1000]:
            lens = rng.integers(0, lenhi, size=n)
            off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
            assert np.array_equal(minimize_order(off), O.minimize_order(off)), (n, lenhi)


def test_no_environment_reads_on_calls():
    """Production behaviour does not depend on the process environment: the
    only getenv calls are sg_ctx_create's seeding of the diagnostics options
    (sg_ctx_set_option sets the rest)."""
    csrc = os.path.join(ROOT, "syzkaller_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        src = open(os.path.join(csrc, f)).read()
        if f != "sg_ctx.hip":
            assert "getenv" not in src, f
            continue
        body = src[src.index("int sg_ctx_create("):]
        body = body[: body.index("\n}\n")]
        assert src.count("getenv") == body.count("getenv") == 3


@pytest.mark.gpu
def test_context_options(ctx):
    from syzkaller_amd._lib import SG_EINVAL, SyzSigError

    assert ctx.get_option("fold_map") == -1 and ctx.get_option("minimize_filter") == 1
    assert ctx.get_option("max_launch_records") == 1 << 24
    ctx.set_option("rpc_decode_blocks", 1)
    assert ctx.get_option("rpc_decode_blocks") == 1
    ctx.set_option("rpc_decode_blocks", -1)
    assert ctx.get_option("m0_filter") == -1
    for bad in (("no_such_option", 1), ("max_launch_records", (1 << 24) + 1), ("max_launch_records", -2),
                ("m0_filter", 2), ("m0_filter", -2), ("prefix_pairs", -1), ("host_copy_threads", 65)):
        with pytest.raises(SyzSigError) as e:
            ctx.set_option(*bad)
        assert e.value.rc == SG_EINVAL
    assert ctx.counter("cpu_quota_milli") >= 1000
