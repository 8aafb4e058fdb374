"""ctypes view of the C ABI in include/hlc.h and the loader for the in-tree libhlc.so.

The library is the product: a HIP (gfx950) build.  There is no CPU fallback -- if the
shared object is missing or cannot be loaded the import of the GPU entry points fails
loudly (`HlcUnavailable`).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref
from ctypes import POINTER, c_char_p, c_double, c_int, c_uint8, c_uint32, c_uint64, c_void_p

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.environ.get("HLC_LIB") or os.path.join(PKG_ROOT, "lib", "libhlc.so")

HLC_NFIELDS = 5
F_OWNER, F_PARENT, F_RECEIVED, F_VOTE_HASH, F_SIGNATURE = range(5)


class HlcUnavailable(RuntimeError):
    pass


class HlcError(RuntimeError):
    pass


class hlc_votes(ctypes.Structure):
    _fields_ = [
        ("n", c_uint64),
        ("vote_id", POINTER(c_uint32)),
        ("proposal_id", POINTER(c_uint32)),
        ("timestamp", POINTER(c_uint64)),
        ("vote", POINTER(c_uint8)),
        ("bytes", POINTER(c_uint8)),
        ("bytes_len", c_uint64),
        ("field_off", POINTER(c_uint64)),
        ("field_len", POINTER(c_uint32)),
    ]


class hlc_proposal(ctypes.Structure):
    _fields_ = [
        ("vote_begin", c_uint64),
        ("vote_count", c_uint32),
        ("proposal_id", c_uint32),
        ("timestamp", c_uint64),
        ("expiration_timestamp", c_uint64),
        ("expected_voters_count", c_uint32),
        ("max_rounds", c_uint32),
        ("consensus_threshold", c_double),
        ("use_gossipsub_rounds", c_uint8),
        ("liveness_criteria_yes", c_uint8),
        ("_pad", c_uint8 * 6),
    ]


class hlc_result(ctypes.Structure):
    _fields_ = [
        ("status", c_uint8),
        ("transition", c_uint8),
        ("scheme_reason", c_uint8),
        ("_pad", c_uint8),
        ("bad_index", c_uint32),
        ("yes", c_uint32),
        ("total", c_uint32),
    ]


class hlc_session_tally(ctypes.Structure):
    _fields_ = [
        ("total", c_uint32),
        ("yes", c_uint32),
        ("expected_voters_count", c_uint32),
        ("state", c_uint8),
        ("liveness_criteria_yes", c_uint8),
        ("_pad", c_uint8 * 2),
        ("consensus_threshold", c_double),
    ]


assert ctypes.sizeof(hlc_session_tally) == 24
assert ctypes.sizeof(hlc_proposal) == 56
assert ctypes.sizeof(hlc_result) == 16

# numpy structured dtypes with the same layout (for zero-copy packing)
try:
    import numpy as np

    PROPOSAL_DTYPE = np.dtype([
        ("vote_begin", "<u8"), ("vote_count", "<u4"), ("proposal_id", "<u4"),
        ("timestamp", "<u8"), ("expiration_timestamp", "<u8"),
        ("expected_voters_count", "<u4"), ("max_rounds", "<u4"),
        ("consensus_threshold", "<f8"), ("use_gossipsub_rounds", "u1"),
        ("liveness_criteria_yes", "u1"), ("_pad", "u1", (6,)),
    ])
    SESSION_TALLY_DTYPE = np.dtype([
        ("total", "<u4"), ("yes", "<u4"), ("expected_voters_count", "<u4"), ("state", "u1"),
        ("liveness_criteria_yes", "u1"), ("_pad", "u1", (2,)), ("consensus_threshold", "<f8"),
    ])
    assert SESSION_TALLY_DTYPE.itemsize == 24
    RESULT_DTYPE = np.dtype([
        ("status", "u1"), ("transition", "u1"), ("scheme_reason", "u1"), ("_pad", "u1"),
        ("bad_index", "<u4"), ("yes", "<u4"), ("total", "<u4"),
    ])
    assert PROPOSAL_DTYPE.itemsize == 56 and RESULT_DTYPE.itemsize == 16
    # hlc_scope_config / hlc_wire_proposal (include/hlc.h, wire decode)
    SCOPE_CONFIG_DTYPE = np.dtype([
        ("consensus_threshold", "<f8"), ("max_rounds", "<u4"), ("use_gossipsub_rounds", "u1"),
        ("_pad", "u1", (3,)),
    ])
    WIRE_PROPOSAL_DTYPE = np.dtype([
        ("name_off", "<u8"), ("payload_off", "<u8"), ("owner_off", "<u8"),
        ("name_len", "<u4"), ("payload_len", "<u4"), ("owner_len", "<u4"), ("round", "<u4"),
        ("bad_vote", "<u4"), ("decode_status", "u1"), ("_pad", "u1", (3,)),
    ])
    assert SCOPE_CONFIG_DTYPE.itemsize == 16 and WIRE_PROPOSAL_DTYPE.itemsize == 48
    # hlc_session (include/hlc.h, streaming votes)
    SESSION_DTYPE = np.dtype([
        ("timestamp", "<u8"), ("expiration_timestamp", "<u8"), ("proposal_id", "<u4"),
        ("expected_voters_count", "<u4"), ("round", "<u4"), ("total", "<u4"), ("yes", "<u4"),
        ("max_rounds", "<u4"), ("consensus_threshold", "<f8"), ("state", "u1"), ("use_gossipsub_rounds", "u1"),
        ("liveness_criteria_yes", "u1"), ("_pad", "u1", (5,)),
    ])
    assert SESSION_DTYPE.itemsize == 56
except ImportError:  # pragma: no cover
    np = None

EXPORTED_SYMBOLS = (
    "hlc_ctx_create", "hlc_ctx_destroy", "hlc_ctx_reserve", "hlc_last_error", "hlc_abi_version",
    "hlc_compute_vote_hashes", "hlc_eth_verify_batch", "hlc_validate_proposals",
    "hlc_validate_proposals_device", "hlc_eth_address_batch", "hlc_eth_sign_batch",
    "hlc_ctx_set_kernel_timing", "hlc_ctx_take_kernel_time", "hlc_ctx_take_chain_time", "hlc_consensus_timeout_batch",
    "hlc_decode_proposals", "hlc_validate_wire_proposals", "hlc_validate_wire_proposals_device",
    "hlc_process_votes", "hlc_process_votes_device", "hlc_synth_arena_bytes", "hlc_synth_votes_device",
    "hlc_synth_byzantine_device", "hlc_outcome_counts_device", "hlc_host_alloc", "hlc_host_free",
    "hlc_host_threads", "hlc_ctx_last_host_trace", "hlc_ctx_set_clock_probe", "hlc_ctx_clock_probe",
    "hlc_validate_proposals_verdicts", "hlc_validate_proposals_verdicts_device", "hlc_encode_vote_payloads",
    "hlc_process_votes_verdicts", "hlc_ctx_set_option", "hlc_ctx_get_option",
)

# hlc_ctx_set_option / hlc_ctx_get_option (include/hlc.h HLC_OPT_*): the host-buffer entries' tunables
OPTIONS = {
    "host_threads": 1, "pool_bind": 2, "nt_copy": 3, "split_votes": 4, "host_trace": 5, "first_batch": 6,
    "rest_pieces": 7, "wire_split_bytes": 8, "wire_front_cap": 9, "wire_chunk": 10, "rec_force_exact": 11,
    "serial_stages": 12, "wire_pipeline": 13, "wire_walk": 14, "split_votes_append": 15,
    "wire_split_bytes_append": 16, "early_comb": 17,
}
LIST_OPTIONS = {"split_votes": "split_votes_append", "wire_split_bytes": "wire_split_bytes_append"}
POOL_BIND_NONE, POOL_BIND_GPU, POOL_BIND_SOURCE = 0, 1, 2

# ConsensusSignatureScheme::verify outcomes as the ABI codes them (include/hlc.h)
VERIFY_TRUE, VERIFY_FALSE, SCHEME_PLUGIN = 0, 1, 7
VERIFY_ERR = 1 + SCHEME_PLUGIN

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libhlc.so and declare the prototypes.  Raises HlcUnavailable if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HlcUnavailable(
            f"libhlc.so not found at {path}; run `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    vp = c_void_p
    u8p = POINTER(c_uint8)
    u32p = POINTER(c_uint32)
    u64p = POINTER(c_uint64)
    lib.hlc_ctx_create.argtypes = [c_int, POINTER(vp)]
    lib.hlc_ctx_create.restype = c_int
    lib.hlc_ctx_destroy.argtypes = [vp]
    lib.hlc_ctx_destroy.restype = None
    lib.hlc_ctx_reserve.argtypes = [vp, c_uint64, c_uint64, c_uint64]
    lib.hlc_ctx_reserve.restype = c_int
    lib.hlc_last_error.argtypes = []
    lib.hlc_last_error.restype = c_char_p
    lib.hlc_abi_version.argtypes = []
    lib.hlc_abi_version.restype = c_int
    lib.hlc_host_alloc.argtypes = [c_uint64, POINTER(c_void_p)]
    lib.hlc_host_alloc.restype = c_int
    lib.hlc_host_free.argtypes = [c_void_p]
    lib.hlc_host_free.restype = None
    lib.hlc_host_threads.argtypes = []
    lib.hlc_host_threads.restype = c_int
    lib.hlc_ctx_last_host_trace.argtypes = [vp]
    lib.hlc_ctx_last_host_trace.restype = c_char_p
    lib.hlc_compute_vote_hashes.argtypes = [vp, POINTER(hlc_votes), u8p]
    lib.hlc_compute_vote_hashes.restype = c_int
    lib.hlc_eth_verify_batch.argtypes = [vp, c_uint64, u8p, c_uint64, u64p, u32p, u64p, u32p,
                                         u64p, u32p, u8p, u8p]
    lib.hlc_eth_verify_batch.restype = c_int
    lib.hlc_validate_proposals.argtypes = [vp, POINTER(hlc_votes), POINTER(hlc_proposal), c_uint64,
                                           c_uint64, POINTER(hlc_result), u8p, u8p, u8p]
    lib.hlc_validate_proposals.restype = c_int
    lib.hlc_validate_proposals_device.argtypes = [vp, POINTER(hlc_votes), POINTER(hlc_proposal),
                                                  c_uint64, c_uint64, POINTER(hlc_result), u8p,
                                                  u8p, u8p, vp]
    lib.hlc_validate_proposals_device.restype = c_int
    lib.hlc_eth_address_batch.argtypes = [vp, c_uint64, u8p, u8p]
    lib.hlc_eth_address_batch.restype = c_int
    lib.hlc_eth_sign_batch.argtypes = [vp, c_uint64, u8p, u8p, c_uint64, u64p, u32p, u8p]
    lib.hlc_eth_sign_batch.restype = c_int
    lib.hlc_consensus_timeout_batch.argtypes = [vp, c_uint64, vp, u8p, u8p]
    lib.hlc_consensus_timeout_batch.restype = c_int
    lib.hlc_decode_proposals.argtypes = [vp, u8p, c_uint64, u64p, u32p, c_uint64, vp, c_uint64, vp, vp,
                                         u64p, u32p, u32p, u64p, u8p, u64p, u32p]
    lib.hlc_decode_proposals.restype = c_int
    lib.hlc_validate_wire_proposals.argtypes = [vp, u8p, c_uint64, u64p, u32p, c_uint64, vp, c_uint64,
                                                c_uint64, vp, vp, u64p]
    lib.hlc_validate_wire_proposals.restype = c_int
    lib.hlc_validate_wire_proposals_device.argtypes = [vp, vp, c_uint64, vp, vp, c_uint64, vp, c_uint64,
                                                       c_uint64, vp, vp, vp]
    lib.hlc_validate_wire_proposals_device.restype = c_int
    lib.hlc_process_votes.argtypes = [vp, POINTER(hlc_votes), u32p, vp, c_uint64, u8p, u32p, c_uint64, c_uint64,
                                      u8p, u8p, u8p, u8p]
    lib.hlc_process_votes.restype = c_int
    lib.hlc_process_votes_device.argtypes = [vp, POINTER(hlc_votes), vp, vp, c_uint64, vp, vp, c_uint64, c_uint64,
                                             vp, vp, vp, vp, vp]
    lib.hlc_process_votes_device.restype = c_int
    lib.hlc_synth_arena_bytes.argtypes = [c_uint64, c_uint32]
    lib.hlc_synth_arena_bytes.restype = c_uint64
    lib.hlc_synth_votes_device.argtypes = [vp, c_uint64, c_uint64, c_uint64, c_uint32, c_uint32, c_int,
                                           POINTER(hlc_votes), vp, vp, vp]
    lib.hlc_synth_votes_device.restype = c_int
    lib.hlc_synth_byzantine_device.argtypes = [vp, c_uint64, c_uint64, c_uint64, c_uint32, POINTER(hlc_votes), vp, vp]
    lib.hlc_synth_byzantine_device.restype = c_int
    lib.hlc_outcome_counts_device.argtypes = [vp, vp, c_uint64, vp, c_uint64, vp, vp]
    lib.hlc_outcome_counts_device.restype = c_int
    lib.hlc_ctx_set_kernel_timing.argtypes = [vp, c_int]
    lib.hlc_ctx_set_kernel_timing.restype = c_int
    lib.hlc_ctx_take_kernel_time.argtypes = [vp, POINTER(ctypes.c_double), u64p, POINTER(ctypes.c_double), u64p]
    lib.hlc_ctx_take_kernel_time.restype = c_int
    lib.hlc_ctx_take_chain_time.argtypes = [vp, POINTER(ctypes.c_double), u64p]
    lib.hlc_ctx_take_chain_time.restype = c_int
    lib.hlc_ctx_set_option.argtypes = [vp, c_int, ctypes.c_int64]
    lib.hlc_ctx_set_option.restype = c_int
    lib.hlc_ctx_get_option.argtypes = [vp, c_int, POINTER(ctypes.c_int64)]
    lib.hlc_ctx_get_option.restype = c_int
    lib.hlc_validate_proposals_verdicts.argtypes = [vp, POINTER(hlc_votes), POINTER(hlc_proposal), c_uint64,
                                                    c_uint64, u8p, POINTER(hlc_result), u8p, u8p]
    lib.hlc_validate_proposals_verdicts.restype = c_int
    lib.hlc_validate_proposals_verdicts_device.argtypes = [vp, POINTER(hlc_votes), POINTER(hlc_proposal), c_uint64,
                                                           c_uint64, vp, vp, vp, vp, vp]
    lib.hlc_validate_proposals_verdicts_device.restype = c_int
    lib.hlc_encode_vote_payloads.argtypes = [vp, POINTER(hlc_votes), u64p, u32p, u8p, c_uint64, u64p]
    lib.hlc_encode_vote_payloads.restype = c_int
    lib.hlc_process_votes_verdicts.argtypes = [vp, POINTER(hlc_votes), u32p, vp, c_uint64, u8p, c_uint64, u64p, u32p,
                                               u32p, c_uint64, c_uint64, u8p, u8p, u8p, u8p, u8p]
    lib.hlc_process_votes_verdicts.restype = c_int
    if hasattr(lib, "hlc_ctx_set_clock_probe"):  # (diagnostics: absent from older builds loaded for A/B runs)
        lib.hlc_ctx_set_clock_probe.argtypes = [vp, c_int]
        lib.hlc_ctx_set_clock_probe.restype = c_int
        lib.hlc_ctx_clock_probe.argtypes = [vp, POINTER(ctypes.c_double), POINTER(ctypes.c_double),
                                            POINTER(ctypes.c_double), u64p]
        lib.hlc_ctx_clock_probe.restype = c_int
    _lib = lib
    return lib


# Every live context owner (engine.Engine): destroyed by an atexit hook, so that no libhlc context --
# its streams, events, device / page-locked buffers and the parked threads of its host staging pool --
# is left for the process's library finalizers (__cxa_finalize of libhlc and the HIP runtime) to
# tear down in an unspecified order (a SIGSEGV inside __cxa_finalize after the
# outputs were written, under rocprofv3).  Python's atexit hooks run before those finalizers.
_live = weakref.WeakSet()


def register_owner(obj) -> None:
    """Adds an object with a close() method to the set destroyed at interpreter exit."""
    _live.add(obj)


@atexit.register
def _close_live_owners() -> None:
    for obj in list(_live):
        try:
            obj.close()
        except Exception:  # noqa: BLE001 -- best effort at exit
            pass


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.hlc_last_error().decode(errors="replace") if _lib is not None else ""
        raise HlcError(f"libhlc call failed with {rc}: {msg}")


def ptr(arr, ctype):
    """ctypes pointer to a numpy array's data (None for None)."""
    if arr is None:
        return None
    return arr.ctypes.data_as(POINTER(ctype))


class _HostBlock:
    """One hlc_host_alloc block; freed when the last reference goes.  It references nothing that
    references it back, so the free happens by reference counting, not at a garbage-collection pass."""

    def __init__(self, lib, nbytes: int):
        self._lib = lib
        self.p = c_void_p()
        check(lib.hlc_host_alloc(max(int(nbytes), 1), ctypes.byref(self.p)))

    def free(self):
        if self.p is not None and self.p.value:
            self._lib.hlc_host_free(self.p)
        self.p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedArena:
    """Page-locked host memory from hlc_host_alloc, handed out as numpy arrays (`take`): input
    arrays built here reach the device without the host-buffer entries' staging copy.  The block is
    freed when the arena and every array taken from it are gone (each array's base chain holds the
    block, not the arena: no reference cycle); an explicit close() frees it at once (only
    when none of its arrays is used again)."""

    def __init__(self, nbytes: int):
        import numpy as np
        self._lib = load_library()
        self.nbytes = int(nbytes)
        self._block = _HostBlock(self._lib, self.nbytes)
        self._p = self._block.p
        buf = (ctypes.c_uint8 * max(self.nbytes, 1)).from_address(self._p.value)
        buf._owner = self._block  # the arrays' base chain keeps the block (not the arena) alive
        self._u8 = np.frombuffer(buf, dtype=np.uint8)
        self._used = 0

    def take(self, shape, dtype):
        """A zeroed array of `shape` / `dtype` carved out of the arena (64-byte aligned)."""
        import numpy as np
        dt = np.dtype(dtype)
        count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
        start = (self._used + 63) & ~63
        end = start + count * dt.itemsize
        if end > self.nbytes:
            raise MemoryError("PinnedArena exhausted")
        self._used = end
        a = self._u8[start:end].view(dt).reshape(shape)
        a[...] = 0
        return a

    def close(self):
        self._block.free()
        self._p = None
