"""Engine: a device context of libhlc.so with numpy-level batch entry points.

Every call goes through the C ABI of include/hlc.h into the gfx950 kernels; nothing here
computes a hash, a signature or a consensus outcome on the CPU.
"""
from __future__ import annotations

import ctypes
import threading
from ctypes import c_uint8, c_uint32, c_uint64, c_void_p
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _ffi
from .batch import VoteBatch, proposals_ptr, results_ptr


def _arena(chunks: Sequence[bytes]):
    lens = np.fromiter((len(c) for c in chunks), dtype=np.uint32, count=len(chunks))
    off = np.zeros(len(chunks), dtype=np.uint64)
    if len(chunks):
        off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    data = b"".join(chunks)
    arena = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
    return arena, off, lens, len(data)


class Engine:
    """One libhlc context on HIP device `device` (default 0)."""

    _default: Optional["Engine"] = None
    _lock = threading.Lock()

    def __init__(self, device: int = 0):
        self.lib = _ffi.load_library()
        h = c_void_p()
        _ffi.check(self.lib.hlc_ctx_create(device, ctypes.byref(h)))
        self.ctx = h
        self.device = device
        _ffi.register_owner(self)  # destroyed at interpreter exit if the caller never closes it

    @classmethod
    def default(cls) -> "Engine":
        """Process-global lazily-initialised context: what the static `Signer::verify` of
        signing.rs:69 needs (no instance is available at the call site)."""
        with cls._lock:
            if cls._default is None:
                cls._default = Engine(0)
            return cls._default

    def close(self) -> None:
        ctx, self.ctx = getattr(self, "ctx", None), None
        if ctx:
            self.lib.hlc_ctx_destroy(ctx)

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, name: str, value) -> None:
        """hlc_ctx_set_option: one of _ffi.OPTIONS (the host-buffer entries' tunables) on this context.  The
        range-size lists (split_votes, wire_split_bytes) also take a sequence or an "a,b,..." string."""
        if name in _ffi.LIST_OPTIONS and not isinstance(value, (int, np.integer)):
            sizes = [int(x) for x in (value.split(",") if isinstance(value, str) else value)]
            _ffi.check(self.lib.hlc_ctx_set_option(self.ctx, _ffi.OPTIONS[name], sizes[0]))
            for x in sizes[1:]:
                _ffi.check(self.lib.hlc_ctx_set_option(self.ctx, _ffi.OPTIONS[_ffi.LIST_OPTIONS[name]], x))
            return
        _ffi.check(self.lib.hlc_ctx_set_option(self.ctx, _ffi.OPTIONS[name], int(value)))

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64(0)
        _ffi.check(self.lib.hlc_ctx_get_option(self.ctx, _ffi.OPTIONS[name], ctypes.byref(v)))
        return int(v.value)

    def options(self, **kv):
        """Context manager: the given options set for the block, restored after it (a range-size list to
        the library default)."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_option(k) for k in kv}
            try:
                for k, v in kv.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, -1 if k in _ffi.LIST_OPTIONS else v)
        return cm()

    def reserve(self, max_votes: int, max_proposals: int, max_bytes: int = 0) -> None:
        _ffi.check(self.lib.hlc_ctx_reserve(self.ctx, max_votes, max_proposals, max_bytes))

    # ---- hot path ---------------------------------------------------------------------
    def validate_proposals(self, batch: VoteBatch, desc: np.ndarray, now: int,
                           want_votes: bool = True, want_recovered: bool = False):
        """hlc_validate_proposals -> (results[np] structured, vote_status[n], vote_reason[n],
        recovered[n,20] or None)."""
        n = batch.n
        res = np.zeros(desc.shape[0], dtype=_ffi.RESULT_DTYPE)
        vst = np.zeros(max(n, 1), np.uint8) if want_votes else None
        vrs = np.zeros(max(n, 1), np.uint8) if want_votes else None
        rec = np.zeros((max(n, 1), 20), np.uint8) if want_recovered else None
        view = batch.view()
        desc = np.ascontiguousarray(desc)
        _ffi.check(self.lib.hlc_validate_proposals(
            self.ctx, ctypes.byref(view), proposals_ptr(desc), desc.shape[0], now, results_ptr(res),
            _ffi.ptr(vst, c_uint8), _ffi.ptr(vrs, c_uint8), _ffi.ptr(rec, c_uint8)))
        return (res, vst[:n] if vst is not None else None, vrs[:n] if vrs is not None else None,
                rec[:n] if rec is not None else None)

    # ---- any ConsensusSignatureScheme (service.rs:39-51): the caller's verdicts -------------------
    def encode_vote_payloads(self, batch: VoteBatch) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """hlc_encode_vote_payloads: the payload Signer::verify gets per vote (utils.rs:150-152, the prost
        encoding with the signature cleared), built on the device -> (arena u8, off u64[n], len u32[n])."""
        n = batch.n
        off = np.zeros(max(n, 1), np.uint64)
        lens = np.zeros(max(n, 1), np.uint32)
        total = c_uint64(0)
        view = batch.view()
        _ffi.check(self.lib.hlc_encode_vote_payloads(self.ctx, ctypes.byref(view), _ffi.ptr(off, c_uint64),
                                                     _ffi.ptr(lens, c_uint32), None, 0, ctypes.byref(total)))
        arena = np.zeros(max(int(total.value), 1), np.uint8)
        _ffi.check(self.lib.hlc_encode_vote_payloads(self.ctx, ctypes.byref(view), _ffi.ptr(off, c_uint64),
                                                     _ffi.ptr(lens, c_uint32), _ffi.ptr(arena, c_uint8), arena.size,
                                                     ctypes.byref(total)))
        return arena[:int(total.value)], off[:n], lens[:n]

    def validate_proposals_verdicts(self, batch: VoteBatch, desc: np.ndarray, now: int, verdicts: np.ndarray,
                                    want_votes: bool = True):
        """hlc_validate_proposals_verdicts: validate-many with the scheme step given per vote by the caller
        (HLC_VERIFY_TRUE / _FALSE / _ERR) -> (results[np], vote_status[n], vote_reason[n])."""
        n = batch.n
        verdicts = np.ascontiguousarray(verdicts, dtype=np.uint8).reshape(-1)
        if verdicts.shape[0] != n:
            raise ValueError(f"verdicts has {verdicts.shape[0]} entries for {n} votes")
        res = np.zeros(desc.shape[0], dtype=_ffi.RESULT_DTYPE)
        vst = np.zeros(max(n, 1), np.uint8) if want_votes else None
        vrs = np.zeros(max(n, 1), np.uint8) if want_votes else None
        view = batch.view()
        desc = np.ascontiguousarray(desc)
        vbuf = verdicts if n else np.zeros(1, np.uint8)
        _ffi.check(self.lib.hlc_validate_proposals_verdicts(
            self.ctx, ctypes.byref(view), proposals_ptr(desc), desc.shape[0], now, _ffi.ptr(vbuf, c_uint8),
            results_ptr(res), _ffi.ptr(vst, c_uint8), _ffi.ptr(vrs, c_uint8)))
        return res, vst[:n] if vst is not None else None, vrs[:n] if vrs is not None else None

    def validate_proposals_verdicts_device(self, dbatch, verdicts_ptr: int, stream_handle: int = 0) -> None:
        """hlc_validate_proposals_verdicts_device on a device.DeviceBatch (verdicts: raw device pointer)."""
        vp = lambda p: ctypes.cast(p, c_void_p)  # noqa: E731
        _ffi.check(self.lib.hlc_validate_proposals_verdicts_device(
            self.ctx, ctypes.byref(dbatch.view), ctypes.cast(dbatch.props_ptr, ctypes.POINTER(_ffi.hlc_proposal)),
            dbatch.n_proposals, dbatch.now, c_void_p(verdicts_ptr), vp(dbatch.results_ptr), vp(dbatch.status_ptr),
            vp(dbatch.reason_ptr), c_void_p(stream_handle) if stream_handle else None))

    def process_votes_verdicts(self, batch: VoteBatch, vote_session: np.ndarray, sessions: np.ndarray,
                               owners: Sequence[bytes], owner_session: np.ndarray, now: int, verdicts: np.ndarray):
        """hlc_process_votes_verdicts: process_incoming_vote (service.rs:286-305) for every vote, in order,
        with the caller's scheme verdicts and owner maps of any identity length.  `sessions` (SESSION_DTYPE)
        is updated in place.  -> (status, transition, inserted, reason)."""
        n = batch.n
        vote_session = np.ascontiguousarray(vote_session, dtype=np.uint32)
        verdicts = np.ascontiguousarray(verdicts, dtype=np.uint8).reshape(-1)
        if verdicts.shape[0] != n or vote_session.shape[0] != n:
            raise ValueError("verdicts / vote_session must have one entry per vote")
        assert sessions.dtype == _ffi.SESSION_DTYPE and sessions.flags.c_contiguous
        oarena, ooff, olen, ototal = _arena(list(owners))
        osess = np.ascontiguousarray(owner_session, dtype=np.uint32)
        m = len(owners)
        out = [np.zeros(max(n, 1), np.uint8) for _ in range(4)]
        view = batch.view()
        one32, one64 = np.zeros(1, np.uint32), np.zeros(1, np.uint64)
        _ffi.check(self.lib.hlc_process_votes_verdicts(
            self.ctx, ctypes.byref(view), _ffi.ptr(vote_session if n else one32, c_uint32),
            c_void_p(sessions.ctypes.data) if sessions.shape[0] else None, sessions.shape[0],
            _ffi.ptr(oarena, c_uint8), ototal, _ffi.ptr(ooff if m else one64, c_uint64),
            _ffi.ptr(olen if m else one32, c_uint32), _ffi.ptr(osess if m else one32, c_uint32), m, now,
            _ffi.ptr(verdicts if n else np.zeros(1, np.uint8), c_uint8), *[_ffi.ptr(o, c_uint8) for o in out]))
        return tuple(o[:n] for o in out)

    def compute_vote_hashes(self, batch: VoteBatch) -> np.ndarray:
        out = np.zeros((max(batch.n, 1), 32), np.uint8)
        view = batch.view()
        _ffi.check(self.lib.hlc_compute_vote_hashes(self.ctx, ctypes.byref(view), _ffi.ptr(out, c_uint8)))
        return out[:batch.n]

    def eth_verify_batch(self, identities: Sequence[bytes], payloads: Sequence[bytes],
                         signatures: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
        """Batched EthereumConsensusSigner::verify -> (status[n], recovered[n,20])."""
        n = len(identities)
        assert len(payloads) == n and len(signatures) == n
        arena, off, lens, total = _arena(list(identities) + list(payloads) + list(signatures))
        st = np.zeros(max(n, 1), np.uint8)
        addr = np.zeros((max(n, 1), 20), np.uint8)
        io, il = off[:n].copy(), lens[:n].copy()
        po, pl = off[n:2 * n].copy(), lens[n:2 * n].copy()
        so, sl = off[2 * n:].copy(), lens[2 * n:].copy()
        _ffi.check(self.lib.hlc_eth_verify_batch(
            self.ctx, n, _ffi.ptr(arena, c_uint8), total, _ffi.ptr(io, c_uint64), _ffi.ptr(il, c_uint32),
            _ffi.ptr(po, c_uint64), _ffi.ptr(pl, c_uint32), _ffi.ptr(so, c_uint64), _ffi.ptr(sl, c_uint32),
            _ffi.ptr(st, c_uint8), _ffi.ptr(addr, c_uint8)))
        return st[:n], addr[:n]

    def eth_verify_arrays(self, arena: np.ndarray, id_off: np.ndarray, id_len: np.ndarray, pay_off: np.ndarray,
                          pay_len: np.ndarray, sig_off: np.ndarray, sig_len: np.ndarray, want_addr: bool = True,
                          out: Optional[Tuple[np.ndarray, np.ndarray]] = None):
        """hlc_eth_verify_batch over pre-packed arrays (one byte arena, per-item u64 offsets and u32
        lengths, contiguous): no per-item Python work.  -> (status[n], recovered[n,20] or None); `out`
        reuses caller-owned output arrays."""
        # the C ABI reads raw u8 / u64 / u32 arrays: convert (a copy only when needed) and check the
        # per-item arrays agree in length before any pointer crosses
        arena = np.ascontiguousarray(arena, dtype=np.uint8).reshape(-1)
        id_off, pay_off, sig_off = (np.ascontiguousarray(a, dtype=np.uint64).reshape(-1) for a in (id_off, pay_off, sig_off))
        id_len, pay_len, sig_len = (np.ascontiguousarray(a, dtype=np.uint32).reshape(-1) for a in (id_len, pay_len, sig_len))
        n = int(id_off.shape[0])
        if any(a.shape[0] != n for a in (id_len, pay_off, pay_len, sig_off, sig_len)):
            raise ValueError("eth_verify_arrays: per-item arrays differ in length")
        if out is not None and (out[0].dtype != np.uint8 or out[0].size < n or not out[0].flags.c_contiguous or
                                (want_addr and (out[1] is None or out[1].dtype != np.uint8 or out[1].size < 20 * n
                                                or not out[1].flags.c_contiguous))):
            raise ValueError("eth_verify_arrays: `out` must be contiguous u8 arrays of n and n x 20")
        if out is None:
            st = np.zeros(max(n, 1), np.uint8)
            addr = np.zeros((max(n, 1), 20), np.uint8) if want_addr else None
        else:
            st, addr = out
        _ffi.check(self.lib.hlc_eth_verify_batch(
            self.ctx, n, _ffi.ptr(arena, c_uint8), int(arena.size), _ffi.ptr(id_off, c_uint64),
            _ffi.ptr(id_len, c_uint32), _ffi.ptr(pay_off, c_uint64), _ffi.ptr(pay_len, c_uint32),
            _ffi.ptr(sig_off, c_uint64), _ffi.ptr(sig_len, c_uint32), _ffi.ptr(st, c_uint8),
            _ffi.ptr(addr, c_uint8) if want_addr else None))
        return st[:n], (addr[:n] if addr is not None else None)

    def consensus_timeout_batch(self, sessions: np.ndarray):
        """hlc_consensus_timeout_batch over a SESSION_TALLY_DTYPE array -> (new state u8[n],
        status u8[n]) -- handle_consensus_timeout (service.rs:323-373) per session."""
        sessions = np.ascontiguousarray(sessions, dtype=_ffi.SESSION_TALLY_DTYPE)
        n = sessions.shape[0]
        state = np.zeros(max(n, 1), np.uint8)
        status = np.zeros(max(n, 1), np.uint8)
        _ffi.check(self.lib.hlc_consensus_timeout_batch(self.ctx, n, c_void_p(sessions.ctypes.data) if n else None,
                                                        _ffi.ptr(state, c_uint8), _ffi.ptr(status, c_uint8)))
        return state[:n], status[:n]

    # ---- streaming votes -----------------------------------------------------------------
    def process_votes(self, batch: VoteBatch, vote_session: np.ndarray, sessions: np.ndarray,
                      owners: Optional[np.ndarray] = None, owner_session: Optional[np.ndarray] = None, now: int = 0):
        """hlc_process_votes: process_incoming_vote (service.rs:286-305) for every vote, in order.
        `sessions` (SESSION_DTYPE) is updated in place.  -> (status, transition, inserted, reason)."""
        n = batch.n
        vote_session = np.ascontiguousarray(vote_session, dtype=np.uint32)
        assert sessions.dtype == _ffi.SESSION_DTYPE and sessions.flags.c_contiguous
        owners = np.zeros((0, 20), np.uint8) if owners is None else np.ascontiguousarray(owners, np.uint8).reshape(-1, 20)
        owner_session = (np.zeros(0, np.uint32) if owner_session is None
                         else np.ascontiguousarray(owner_session, dtype=np.uint32))
        out = [np.zeros(max(n, 1), np.uint8) for _ in range(4)]
        view = batch.view()
        obuf = owners if owners.size else np.zeros((1, 20), np.uint8)
        osb = owner_session if owner_session.size else np.zeros(1, np.uint32)
        _ffi.check(self.lib.hlc_process_votes(
            self.ctx, ctypes.byref(view), _ffi.ptr(vote_session if n else np.zeros(1, np.uint32), c_uint32),
            c_void_p(sessions.ctypes.data) if sessions.shape[0] else None, sessions.shape[0],
            _ffi.ptr(obuf, c_uint8), _ffi.ptr(osb, c_uint32), owners.shape[0], now,
            *[_ffi.ptr(o, c_uint8) for o in out]))
        return tuple(o[:n] for o in out)

    def process_votes_device(self, dbatch, vote_session_ptr: int, sessions_ptr: int, n_sessions: int, now: int,
                             st_ptr: int, tr_ptr: int, ins_ptr: int, stream_handle: int = 0) -> None:
        """hlc_process_votes_device: votes of a device.DeviceBatch, session arrays and outputs in HBM
        (raw device pointers as ints); no existing owner maps."""
        _ffi.check(self.lib.hlc_process_votes_device(
            self.ctx, ctypes.byref(dbatch.view), c_void_p(vote_session_ptr), c_void_p(sessions_ptr), n_sessions,
            None, None, 0, now, c_void_p(st_ptr), c_void_p(tr_ptr), c_void_p(ins_ptr), None,
            c_void_p(stream_handle) if stream_handle else None))

    # ---- wire format (gossip bytes of consensus.proto Proposal messages) -----------------
    @staticmethod
    def _wire_args(wire, msg_off, msg_len, scope):
        wire = np.ascontiguousarray(np.frombuffer(wire, np.uint8) if isinstance(wire, (bytes, bytearray)) else wire,
                                    dtype=np.uint8)
        msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
        msg_len = np.ascontiguousarray(msg_len, dtype=np.uint32)
        scope = np.ascontiguousarray(scope, dtype=_ffi.SCOPE_CONFIG_DTYPE).reshape(-1)
        buf = wire if wire.size else np.zeros(1, np.uint8)
        return buf, int(wire.size), msg_off, msg_len, scope

    def decode_proposals(self, wire, msg_off, msg_len, scope):
        """hlc_decode_proposals -> (props PROPOSAL_DTYPE[m], wire_info WIRE_PROPOSAL_DTYPE[m],
        VoteBatch of the decoded votes whose arena is `wire`)."""
        buf, wlen, msg_off, msg_len, scope = self._wire_args(wire, msg_off, msg_len, scope)
        m = msg_off.shape[0]
        props = np.zeros(max(m, 1), _ffi.PROPOSAL_DTYPE)
        winfo = np.zeros(max(m, 1), _ffi.WIRE_PROPOSAL_DTYPE)
        nv = c_uint64(0)
        args = (self.ctx, _ffi.ptr(buf, c_uint8), wlen, _ffi.ptr(msg_off, c_uint64), _ffi.ptr(msg_len, c_uint32), m,
                c_void_p(scope.ctypes.data), scope.shape[0], c_void_p(props.ctypes.data),
                c_void_p(winfo.ctypes.data), ctypes.byref(nv))
        _ffi.check(self.lib.hlc_decode_proposals(*args, None, None, None, None, None, None))  # count only
        n = nv.value
        vid = np.zeros(max(n, 1), np.uint32)
        pid = np.zeros(max(n, 1), np.uint32)
        ts = np.zeros(max(n, 1), np.uint64)
        vt = np.zeros(max(n, 1), np.uint8)
        foff = np.zeros((max(n, 1), 5), np.uint64)
        flen = np.zeros((max(n, 1), 5), np.uint32)
        nv.value = max(n, 1)
        _ffi.check(self.lib.hlc_decode_proposals(*args, _ffi.ptr(vid, c_uint32), _ffi.ptr(pid, c_uint32),
                                                 _ffi.ptr(ts, c_uint64), _ffi.ptr(vt, c_uint8),
                                                 _ffi.ptr(foff, c_uint64), _ffi.ptr(flen, c_uint32)))
        batch = VoteBatch(vote_id=vid[:n], proposal_id=pid[:n], timestamp=ts[:n], vote=vt[:n],
                          arena=buf[:wlen], field_off=foff[:n], field_len=flen[:n])
        return props[:m], winfo[:m], batch

    def validate_wire_proposals(self, wire, msg_off, msg_len, scope, now: int):
        """hlc_validate_wire_proposals (process_incoming_proposal from wire bytes) ->
        (results RESULT_DTYPE[m], wire_info WIRE_PROPOSAL_DTYPE[m], decoded vote count)."""
        buf, wlen, msg_off, msg_len, scope = self._wire_args(wire, msg_off, msg_len, scope)
        m = msg_off.shape[0]
        res = np.zeros(max(m, 1), _ffi.RESULT_DTYPE)
        winfo = np.zeros(max(m, 1), _ffi.WIRE_PROPOSAL_DTYPE)
        nv = c_uint64(0)
        _ffi.check(self.lib.hlc_validate_wire_proposals(
            self.ctx, _ffi.ptr(buf, c_uint8), wlen, _ffi.ptr(msg_off, c_uint64), _ffi.ptr(msg_len, c_uint32), m,
            c_void_p(scope.ctypes.data), scope.shape[0], now, c_void_p(res.ctypes.data),
            c_void_p(winfo.ctypes.data), ctypes.byref(nv)))
        return res[:m], winfo[:m], nv.value

    # ---- signing side -------------------------------------------------------------------
    def address_batch(self, priv: np.ndarray) -> np.ndarray:
        priv = np.ascontiguousarray(priv, dtype=np.uint8).reshape(-1, 32)
        n = priv.shape[0]
        out = np.zeros((max(n, 1), 20), np.uint8)
        _ffi.check(self.lib.hlc_eth_address_batch(self.ctx, n, _ffi.ptr(priv, c_uint8), _ffi.ptr(out, c_uint8)))
        return out[:n]

    def sign_batch(self, priv: np.ndarray, payloads: Sequence[bytes]) -> np.ndarray:
        priv = np.ascontiguousarray(priv, dtype=np.uint8).reshape(-1, 32)
        n = priv.shape[0]
        arena, off, lens, total = _arena(list(payloads))
        return self.sign_batch_arena(priv, arena, off, lens, total)

    def sign_batch_arena(self, priv: np.ndarray, arena: np.ndarray, off: np.ndarray, lens: np.ndarray,
                         total: int) -> np.ndarray:
        n = priv.shape[0]
        out = np.zeros((max(n, 1), 65), np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        _ffi.check(self.lib.hlc_eth_sign_batch(
            self.ctx, n, _ffi.ptr(priv, c_uint8), _ffi.ptr(arena, c_uint8), total, _ffi.ptr(off, c_uint64),
            _ffi.ptr(lens, c_uint32), _ffi.ptr(out, c_uint8)))
        return out[:n]

    # ---- device-resident path (inputs already in HBM) -----------------------------------
    def validate_proposals_device(self, dbatch, stream_handle: int = 0) -> None:
        """hlc_validate_proposals_device over a `device.DeviceBatch` (all pointers in HBM);
        enqueued on `stream_handle` (a hipStream_t as int; 0 = the context's stream)."""
        _ffi.check(self.lib.hlc_validate_proposals_device(
            self.ctx, ctypes.byref(dbatch.view), dbatch.props_ptr, dbatch.n_proposals, dbatch.now,
            dbatch.results_ptr, dbatch.status_ptr, dbatch.reason_ptr, dbatch.recovered_ptr,
            c_void_p(stream_handle) if stream_handle else None))

    def synth_votes_device(self, dbatch, seed: int, start_proposal: int, n_proposals: int, votes_per_proposal: int,
                           expected_voters: int, gossipsub: bool, priv_ptr: int = 0, stream_handle: int = 0) -> None:
        """hlc_synth_votes_device into a `device.DeviceBatch.allocate`d batch (see
        DeviceBatch.synthetic)."""
        _ffi.check(self.lib.hlc_synth_votes_device(
            self.ctx, seed, start_proposal, n_proposals, votes_per_proposal, expected_voters, 1 if gossipsub else 0,
            ctypes.byref(dbatch.view), c_void_p(ctypes.cast(dbatch.props_ptr, c_void_p).value),
            c_void_p(priv_ptr) if priv_ptr else None, c_void_p(stream_handle) if stream_handle else None))

    def synth_byzantine_device(self, dbatch, seed: int, start_proposal: int, n_proposals: int,
                               votes_per_proposal: int, kind_ptr: int, stream_handle: int = 0) -> None:
        """hlc_synth_byzantine_device: the config-5 mutations, in place, over a batch made by
        synth_votes_device with the same arguments; per-vote kinds (HLC_BYZ_*) into kind_ptr."""
        _ffi.check(self.lib.hlc_synth_byzantine_device(
            self.ctx, seed, start_proposal, n_proposals, votes_per_proposal, ctypes.byref(dbatch.view),
            c_void_p(kind_ptr), c_void_p(stream_handle) if stream_handle else None))

    def outcome_counts_device(self, status_ptr: int, n_votes: int, results_ptr: int, n_proposals: int,
                              counts_ptr: int, stream_handle: int = 0) -> None:
        """hlc_outcome_counts_device: u64[64] histograms (votes by status, proposals by status)."""
        _ffi.check(self.lib.hlc_outcome_counts_device(
            self.ctx, c_void_p(status_ptr), n_votes, c_void_p(results_ptr), n_proposals, c_void_p(counts_ptr),
            c_void_p(stream_handle) if stream_handle else None))

    def validate_wire_proposals_device(self, dwire, stream_handle: int = 0) -> None:
        """hlc_validate_wire_proposals_device over a `device.DeviceWire` (wire bytes, message
        extents and scope configs in HBM); results land in dwire.results."""
        _ffi.check(self.lib.hlc_validate_wire_proposals_device(
            self.ctx, dwire.wire_ptr, dwire.wire_len, dwire.off_ptr, dwire.len_ptr, dwire.n_msgs, dwire.scope_ptr,
            dwire.n_scope, dwire.now, dwire.results_ptr, dwire.winfo_ptr,
            c_void_p(stream_handle) if stream_handle else None))

    def last_host_trace(self) -> Optional[dict]:
        """The last host-buffer call's phase times (HLC_HOST_TRACE=1 or 2 in the environment), or None."""
        import json
        raw = self.lib.hlc_ctx_last_host_trace(self.ctx)
        return json.loads(raw.decode()) if raw else None

    def set_kernel_timing(self, enable: bool, recovery_only: bool = False) -> None:
        """Time later validate-many calls with dispatch-bound HIP events: the recovery bracket, and unless
        recovery_only also the chain/tally kernels and the whole call (HLC_TIMING_ALL / HLC_TIMING_RECOVERY)."""
        mode = (2 if recovery_only else 1) if enable else 0
        _ffi.check(self.lib.hlc_ctx_set_kernel_timing(self.ctx, mode))

    def take_kernel_time(self):
        """-> (recover_ms, recover_launches, call_ms, calls) since the previous take."""
        rms, cms = ctypes.c_double(), ctypes.c_double()
        rl, cl = c_uint64(), c_uint64()
        _ffi.check(self.lib.hlc_ctx_take_kernel_time(self.ctx, ctypes.byref(rms), ctypes.byref(rl),
                                                     ctypes.byref(cms), ctypes.byref(cl)))
        return rms.value, rl.value, cms.value, cl.value

    def set_clock_probe(self, enable: bool) -> None:
        """k_rec_main of later validate_proposals_device calls stamps each wave's clock ticks (diagnostic)."""
        _ffi.check(self.lib.hlc_ctx_set_clock_probe(self.ctx, 1 if enable else 0))

    def clock_probe(self) -> dict:
        """The shader clock the last stamped k_rec_main launch's waves ran at (hlc_ctx_clock_probe)."""
        med, lo, hi = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        w = c_uint64()
        _ffi.check(self.lib.hlc_ctx_clock_probe(self.ctx, ctypes.byref(med), ctypes.byref(lo), ctypes.byref(hi),
                                                ctypes.byref(w)))
        return {"median_GHz": med.value, "min_GHz": lo.value, "max_GHz": hi.value, "waves": w.value}

    def take_chain_time(self):
        """-> (chain_ms, launches): chain-check + duplicate + tally kernels since the previous take."""
        ms, n = ctypes.c_double(), c_uint64()
        _ffi.check(self.lib.hlc_ctx_take_chain_time(self.ctx, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value
