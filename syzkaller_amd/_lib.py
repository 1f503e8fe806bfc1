"""ctypes binding of libsyzsig.so (include/syzsig.h).

The library is the product: HIP kernels for gfx950 behind a C-ABI.  There is
no CPU fallback -- if the shared object is missing or no MI355X is present,
calls fail loudly (ImportError here, SyzSigError from compute calls).
"""
import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SG_LIB_PATH") or os.path.join(_HERE, "libsyzsig.so")  # override: diagnostics builds

SG_OK = 0
SG_EINVAL = -1
SG_EHIP = -2
SG_ENOMEM = -3
SG_ENODEV = -4

OP_DIFFERENCE = 0
OP_SYMDIFF = 1
OP_UNION = 2
OP_INTERSECT = 3

P32 = POINTER(c_uint32)
P64 = POINTER(c_uint64)
P8 = POINTER(c_uint8)
PSZ = POINTER(c_size_t)
PINT = POINTER(c_int)

# name -> (restype, argtypes); mirrors include/syzsig.h one to one.
SIGNATURES = {
    "sg_version": (c_char_p, []),
    "sg_last_error": (c_char_p, []),
    "sg_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "sg_ctx_destroy": (None, [c_void_p]),
    "sg_ctx_sync": (c_int, [c_void_p]),
    "sg_ctx_set_stream": (c_int, [c_void_p, c_void_p]),
    "sg_ctx_reset_stream": (c_int, [c_void_p]),
    "sg_ctx_stream": (c_void_p, [c_void_p]),
    "sg_ctx_timing": (c_int, [c_void_p, c_int]),
    "sg_ctx_kernel_time": (c_int, [c_void_p, c_char_p, POINTER(c_double), P64]),
    "sg_ctx_counter": (c_int, [c_void_p, c_char_p, P64]),
    "sg_ctx_set_option": (c_int, [c_void_p, c_char_p, c_int64]),
    "sg_ctx_get_option": (c_int, [c_void_p, c_char_p, POINTER(c_int64)]),
    "sg_ctx_marker": (c_int, [c_void_p, c_int, c_uint32]),
    "sg_set_create": (c_int, [c_void_p, POINTER(c_void_p)]),
    "sg_set_destroy": (None, [c_void_p]),
    "sg_set_clear": (c_int, [c_void_p]),
    "sg_set_count": (c_int, [c_void_p, P64]),
    "sg_set_export": (c_int, [c_void_p, P32, c_size_t, PSZ]),
    "sg_set_add": (c_int, [c_void_p, P32, c_size_t]),
    "sg_set_new": (c_int, [c_void_p, P32, c_size_t, PINT]),
    "sg_set_diff": (c_int, [c_void_p, P32, c_size_t, P32, PSZ]),
    "sg_set_device_words": (c_void_p, [c_void_p]),
    "sg_set_wrap_dev": (c_int, [c_void_p, c_void_p, POINTER(c_void_p)]),
    "sg_set_or_dev": (c_int, [c_void_p, c_void_p]),
    "sg_set_copy": (c_int, [c_void_p, c_void_p]),
    "sg_set_or_new_dev": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sg_set_count_missing_dev": (c_int, [c_void_p, c_void_p, c_uint64, P64]),
    "sg_triage_batch": (c_int, [c_void_p, c_void_p, c_void_p, P32, P64, c_size_t, P8, P32, P64, P64]),
    "sg_triage_batch_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64,
                                    c_void_p, c_void_p, c_void_p]),
    "sg_triage_traces": (c_int, [c_void_p, c_void_p, c_void_p, P32, P64, c_size_t, P8]),
    "sg_triage_traces_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_void_p]),
    "sg_shard_of": (c_int, [c_uint32, c_uint32]),
    "sg_shard_candidates_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64,
                                        c_uint32, c_void_p, c_void_p]),
    "sg_shard_owners_dev": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "sg_shard_flags_dev": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_uint64, c_uint64, c_void_p]),
    "sg_set_add_dev": (c_int, [c_void_p, c_void_p, c_uint64]),
    "sg_set_add_new_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64]),
    "sg_set_del_dev": (c_int, [c_void_p, c_void_p, c_uint64]),
    "sg_prefix_cands_dev": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64]),
    "sg_bitmap_prefix_or_dev": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p]),
    "sg_bitmap_prefix_or_rank_dev": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p]),
    "sg_set_or_new_or_dev": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sg_prefix_begin_dev": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64]),
    "sg_prefix_end_dev": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sg_prefix_flags_dev": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p]),
    "sg_prefix_begin_form_dev": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64,
                                         c_uint64, c_void_p]),
    "sg_add_inputs": (c_int, [c_void_p, c_void_p, c_void_p, P32, P64, c_size_t]),
    "sg_triage_newsig": (c_int, [c_void_p, c_void_p, P32, P64, c_size_t, P32, P64]),
    "sg_triage_intersect": (c_int, [c_void_p, P32, P64, P32, P64, c_size_t, P64]),
    "sg_triage_subset": (c_int, [c_void_p, P32, P64, P32, P64, c_size_t, P8]),
    "sg_accept_batch": (c_int, [c_void_p, c_void_p, c_void_p, P32, P64, P32, P64, c_size_t, P8]),
    "sg_merge_poll": (c_int, [c_void_p, c_void_p, P32, P64, c_size_t, P32, P64]),
    "sg_minimize": (c_int, [c_void_p, P32, P64, c_size_t, P32, P32, PSZ]),
    "sg_minimize_order": (c_int, [P64, c_size_t, P32]),
    "sg_delta_encode_batch": (c_int, [c_void_p, P32, P64, c_size_t, P8, c_size_t, P64]),
    "sg_delta_decode_batch": (c_int, [c_void_p, P8, P64, c_size_t, P32, c_size_t, P64]),
    "sg_set_encode": (c_int, [c_void_p, P8, c_size_t, PSZ]),
    "sg_set_decode_add": (c_int, [c_void_p, P8, c_size_t, P64]),
    "sg_sancov_batch": (c_int, [c_void_p, P32, P64, c_size_t, P8]),
    "sg_canonicalize": (c_int, [c_void_p, P32, c_size_t, PSZ]),
    "sg_canonicalize_batch": (c_int, [c_void_p, P32, P64, c_size_t, P64]),
    "sg_merge": (c_int, [c_void_p, c_int, P32, c_size_t, P32, c_size_t, P32, PSZ]),
    "sg_merge_batch": (c_int, [c_void_p, c_int, P32, c_size_t, P64, P64, P32, c_size_t, P64, P64, c_size_t, P32,
                               c_size_t, P64, P64]),
    "sg_union_fold": (c_int, [c_void_p, P32, P64, c_size_t, P32, c_size_t, P32, c_size_t, P64]),
    "sg_has_difference": (c_int, [c_void_p, P32, c_size_t, P32, c_size_t, PINT]),
    "sg_has_difference_batch": (c_int, [c_void_p, P32, c_size_t, P64, P64, P32, c_size_t, P64, P64, c_size_t,
                                        c_void_p]),
    "sg_exec_signal": (c_int, [c_void_p, P32, P64, P64, c_size_t, P32, P64]),
    "sg_exec_signal_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_void_p,
                                   c_void_p]),
    "sg_exec_signal_queued_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_void_p,
                                          c_void_p, c_void_p]),
    "sg_triage_traces_queued": (c_int, [c_void_p, c_void_p, c_void_p, P32, P64, P64, c_size_t, P8, P32, P64]),
    "sg_gen_zipf_traces_dev": (c_int, [c_void_p, c_uint64, c_uint64, c_double, c_uint32, c_uint64, c_uint64, c_uint32,
                                       c_uint32, c_void_p]),
    "sg_gen_population_traces_dev": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_double, c_double,
                                             c_uint32, c_uint64, c_uint64, c_uint32, c_uint32, c_void_p]),
    "sg_cover_uncovered": (c_int, [c_void_p, P32, c_size_t, c_uint32, P64, P64, c_size_t, P64, c_size_t, P64, PSZ]),
    "sg_ipc_parse": (c_int, [c_void_p, P32, P64, P64, P32, c_size_t, POINTER(c_int64), P8, POINTER(c_int32), P64, P32,
                             P64, P32]),
    "sg_ipc_parse_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
}


class SyzSigError(RuntimeError):
    def __init__(self, fn, rc, msg):
        super().__init__(f"{fn} failed ({rc}): {msg}")
        self.rc = rc


def _preload_torch_hip_runtime():
    """One HIP runtime per process: when PyTorch-ROCm is installed, bind
    libsyzsig to the libamdhip64 that torch ships (torch loads it by the name
    `libamdhip64.so`, we by the soname `libamdhip64.so.7`; loading ours first
    would put two runtimes in the process).  Does not import torch."""
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            rt = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
            if os.path.exists(rt):
                ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)
    except OSError:
        pass


def _load():
    _preload_torch_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C syzkaller_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(fn_name, rc):
    if rc != SG_OK:
        msg = lib.sg_last_error()
        raise SyzSigError(fn_name, rc, msg.decode() if msg else "")
    return rc


def call(fn_name, *args):
    return check(fn_name, getattr(lib, fn_name)(*args))
