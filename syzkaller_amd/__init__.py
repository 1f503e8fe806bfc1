"""syzkaller_amd -- MI355X-native coverage-signal triage engine for syzkaller.

The product is libsyzsig.so (HIP kernels for gfx950 behind the C-ABI in
include/syzsig.h).  `syzkaller_amd.cover` mirrors the reference pkg/cover API
and the fuzzer/manager signal loops on top of it; `syzkaller_amd.shard` runs
one batch's triage hash-sharded by signal across GPUs (RCCL all-to-all), and
`syzkaller_amd.dist` holds the Poll OR-exchange between independent fuzzers.
"""
from ._lib import LIB_PATH, SyzSigError, lib  # noqa: F401  (fails loudly if the library is missing)

__all__ = ["LIB_PATH", "SyzSigError", "lib"]
