"""Device-resident vote batches: the SoA arrays of a VoteBatch uploaded once to HBM (torch
tensors are used only as device-memory plumbing) and an `hlc_votes` view of device pointers
for hlc_validate_proposals_device."""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_uint8, c_uint32, c_uint64

import numpy as np

from . import _ffi
from .batch import VoteBatch


class DeviceBatch:
    """A vote batch + its proposals resident in HBM.  Built from host arrays (`DeviceBatch(batch,
    desc, now)`), or generated on the device (`DeviceBatch.synthetic`: hlc_synth_votes_device, the
    SURVEY §8d workload, so a rank of a sharded run builds only its own shard and nothing crosses
    PCIe)."""

    def __init__(self, batch: VoteBatch, desc: np.ndarray, now: int, device: str = "cuda:0"):
        import torch

        def up(a):
            a = np.ascontiguousarray(a)
            t = torch.from_numpy(a.view(np.uint8).reshape(-1).copy())
            return t.to(device)

        arena = batch.arena if batch.arena.size else np.zeros(1, np.uint8)
        t = {
            "vote_id": up(batch.vote_id), "proposal_id": up(batch.proposal_id), "timestamp": up(batch.timestamp),
            "vote": up(batch.vote), "bytes": up(arena), "field_off": up(batch.field_off),
            "field_len": up(batch.field_len), "props": up(desc),
        }
        self._bind(t, batch.n, int(batch.arena.size), int(desc.shape[0]), now, device)

    @classmethod
    def allocate(cls, n: int, arena_bytes: int, n_proposals: int, now: int, device: str = "cuda:0") -> "DeviceBatch":
        import torch
        self = cls.__new__(cls)

        def z(nbytes):
            return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)

        t = {"vote_id": z(4 * n), "proposal_id": z(4 * n), "timestamp": z(8 * n), "vote": z(n),
             "bytes": z(arena_bytes), "field_off": z(8 * 5 * n), "field_len": z(4 * 5 * n),
             "props": z(_ffi.PROPOSAL_DTYPE.itemsize * n_proposals)}
        self._bind(t, n, int(arena_bytes), n_proposals, now, device)
        return self

    @classmethod
    def synthetic(cls, engine, n_proposals: int, votes_per_proposal: int, expected_voters: int, gossipsub: bool,
                  seed: int, start_proposal: int = 0, device: str = "cuda:0", want_priv: bool = False,
                  stream_handle: int = 0) -> "DeviceBatch":
        """Global proposals [start_proposal, start_proposal + n_proposals) of the synth.py spec,
        generated and signed on the GPU (bit-identical to synth.generate)."""
        from .synth import NOW
        P, V = int(n_proposals), int(votes_per_proposal)
        nbytes = int(engine.lib.hlc_synth_arena_bytes(P, V))
        self = cls.allocate(P * V, nbytes, P, NOW, device)
        self.priv = None
        if want_priv:
            import torch
            self.priv = torch.empty(max(P * V * 32, 1), dtype=torch.uint8, device=device)
        engine.synth_votes_device(self, seed, start_proposal, P, V, expected_voters, gossipsub,
                                  self.priv.data_ptr() if self.priv is not None else 0, stream_handle)
        if not stream_handle:
            # the context's stream does not order with torch's streams: finish before torch reads
            self.torch.cuda.synchronize(device)
        return self

    def make_byzantine(self, engine, seed: int, start_proposal: int = 0) -> np.ndarray:
        """SURVEY.md §8d config 5 on the device: mutate this synthetic batch (made by `synthetic`
        with the same seed / start) into the 1/3-Byzantine mix in place (hlc_synth_byzantine_device)
        and return the per-vote mutation kinds (byzantine.py)."""
        import torch
        V = self.n // max(self.n_proposals, 1)
        kinds = torch.zeros(max(self.n, 1), dtype=torch.uint8, device=self.device)
        engine.synth_byzantine_device(self, seed, start_proposal, self.n_proposals, V, kinds.data_ptr())
        torch.cuda.synchronize(self.device)
        return kinds[: self.n].cpu().numpy()

    def choice_numpy(self) -> np.ndarray:
        return self._t["vote"][: self.n].cpu().numpy()

    def _bind(self, t, n: int, bytes_len: int, n_proposals: int, now: int, device: str) -> None:
        import torch
        self.torch = torch
        self.device = device
        self.n = int(n)
        self.n_proposals = int(n_proposals)
        self.now = int(now)
        self.bytes_len = int(bytes_len)
        self._t = t
        self.results = torch.zeros(self.n_proposals * 16 + 16, dtype=torch.uint8, device=device)
        self.status = torch.zeros(self.n + 1, dtype=torch.uint8, device=device)
        self.reason = torch.zeros(self.n + 1, dtype=torch.uint8, device=device)
        self.recovered = None
        self.view = _ffi.hlc_votes(
            n=self.n,
            vote_id=ctypes.cast(t["vote_id"].data_ptr(), POINTER(c_uint32)),
            proposal_id=ctypes.cast(t["proposal_id"].data_ptr(), POINTER(c_uint32)),
            timestamp=ctypes.cast(t["timestamp"].data_ptr(), POINTER(c_uint64)),
            vote=ctypes.cast(t["vote"].data_ptr(), POINTER(c_uint8)),
            bytes=ctypes.cast(t["bytes"].data_ptr(), POINTER(c_uint8)),
            bytes_len=self.bytes_len,
            field_off=ctypes.cast(t["field_off"].data_ptr(), POINTER(c_uint64)),
            field_len=ctypes.cast(t["field_len"].data_ptr(), POINTER(c_uint32)),
        )
        self.props_ptr = ctypes.cast(t["props"].data_ptr(), POINTER(_ffi.hlc_proposal))
        self.results_ptr = ctypes.cast(self.results.data_ptr(), POINTER(_ffi.hlc_result))
        self.status_ptr = ctypes.cast(self.status.data_ptr(), POINTER(c_uint8))
        self.reason_ptr = ctypes.cast(self.reason.data_ptr(), POINTER(c_uint8))
        self.recovered_ptr = None

    def want_recovered(self) -> None:
        """Allocates the optional per-vote recovered-address output (n x 20 bytes)."""
        if self.recovered is None:
            self.recovered = self.torch.zeros(max(self.n * 20, 1), dtype=self.torch.uint8, device=self.device)
            self.recovered_ptr = ctypes.cast(self.recovered.data_ptr(), POINTER(c_uint8))

    def results_numpy(self) -> np.ndarray:
        raw = self.results[: self.n_proposals * 16].cpu().numpy()
        return raw.view(_ffi.RESULT_DTYPE)

    def status_numpy(self) -> np.ndarray:
        return self.status[: self.n].cpu().numpy()

    def desc_numpy(self) -> np.ndarray:
        return self._t["props"][: self.n_proposals * _ffi.PROPOSAL_DTYPE.itemsize].cpu().numpy().view(
            _ffi.PROPOSAL_DTYPE)

    def to_host(self):
        """The whole batch back on the host: (VoteBatch, desc, priv u8[n,32] or None)."""
        self.torch.cuda.synchronize(self.device)
        t = self._t

        def arr(name, dtype, count, width=1):
            a = t[name][: count * np.dtype(dtype).itemsize * width].cpu().numpy().view(dtype)
            return a.reshape(-1, width) if width > 1 else a

        n = self.n
        batch = VoteBatch(arr("vote_id", np.uint32, n), arr("proposal_id", np.uint32, n),
                          arr("timestamp", np.uint64, n), arr("vote", np.uint8, n),
                          t["bytes"][: self.bytes_len].cpu().numpy(), arr("field_off", np.uint64, n, 5),
                          arr("field_len", np.uint32, n, 5))
        priv = None
        if getattr(self, "priv", None) is not None:
            priv = self.priv[: n * 32].cpu().numpy().reshape(-1, 32)
        return batch, self.desc_numpy().copy(), priv

    def host_prefix(self, p: int):
        """The first `p` proposals with every vote up to their last one and the arena up to the last
        byte those votes reference, copied back to the host: (VoteBatch, desc).  No re-basing -- the
        cheap host sample of a large device-generated shard (bench.py's CPU baseline at N > 1)."""
        self.torch.cuda.synchronize(self.device)
        t = self._t
        desc = self.desc_numpy()[:p].copy()
        nv = int((desc["vote_begin"] + desc["vote_count"]).max()) if p else 0

        def arr(name, dtype, width=1):
            a = t[name][: nv * np.dtype(dtype).itemsize * width].cpu().numpy().view(dtype)
            return a.reshape(-1, width) if width > 1 else a

        foff, flen = arr("field_off", np.uint64, 5), arr("field_len", np.uint32, 5)
        end = int((foff + flen).max()) if nv else 0
        batch = VoteBatch(arr("vote_id", np.uint32), arr("proposal_id", np.uint32), arr("timestamp", np.uint64),
                          arr("vote", np.uint8), t["bytes"][:max(end, 1)].cpu().numpy()[:end], foff, flen)
        return batch, desc

    def host_proposals(self, idx) -> tuple:
        """Proposals `idx` (indices into this batch) with their votes copied back to the host as a
        self-contained (VoteBatch, desc, global vote index) triple -- the CPU cross-check of a
        sample of a device-generated shard.  Each proposal's votes are contiguous."""
        self.torch.cuda.synchronize(self.device)
        t = self._t
        desc_all = self.desc_numpy()
        idx = np.asarray(idx, np.int64)
        sub = desc_all[idx].copy()
        vidx = np.concatenate([np.arange(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"]),
                                         dtype=np.int64) for d in sub]) if idx.size else np.zeros(0, np.int64)
        tv = self.torch.from_numpy(vidx).to(self.device)

        def rows(name, dtype, width=1):
            item = np.dtype(dtype).itemsize * width
            a = t[name][: self.n * item].view(-1, item).index_select(0, tv).cpu().numpy()
            return a.reshape(-1).view(dtype).reshape((-1, width) if width > 1 else (-1,))

        foff = rows("field_off", np.uint64, 5)
        flen = rows("field_len", np.uint32, 5)
        # compact arena: every field of the sampled votes, re-based
        arena_dev = t["bytes"]
        pieces, new_off, pos, cache = [], np.zeros_like(foff), 0, {}
        for k, (o, l) in enumerate(zip(foff.reshape(-1), flen.reshape(-1))):
            o, l = int(o), int(l)
            if not l:
                new_off.reshape(-1)[k] = pos
                continue
            if (o, l) not in cache:
                cache[(o, l)] = pos
                pieces.append((o, l))
                pos += l
            new_off.reshape(-1)[k] = cache[(o, l)]
        if pieces:
            gather = np.concatenate([np.arange(o, o + l, dtype=np.int64) for o, l in pieces])
            arena = arena_dev.index_select(0, self.torch.from_numpy(gather).to(self.device)).cpu().numpy()
        else:
            arena = np.zeros(0, np.uint8)
        begins = np.zeros(sub.shape[0], np.uint64)
        if sub.shape[0]:
            begins[1:] = np.cumsum(sub["vote_count"].astype(np.uint64))[:-1]
        sub["vote_begin"] = begins
        batch = VoteBatch(rows("vote_id", np.uint32), rows("proposal_id", np.uint32), rows("timestamp", np.uint64),
                          rows("vote", np.uint8), arena, new_off.astype(np.uint64), flen.copy())
        return batch, sub, vidx


class DeviceWire:
    """Gossip bytes of n Proposal messages resident in HBM (synth.to_wire layout) for
    hlc_validate_wire_proposals_device."""

    def __init__(self, wire: np.ndarray, msg_off: np.ndarray, msg_len: np.ndarray, scope: np.ndarray, now: int,
                 device: str = "cuda:0"):
        import torch
        from ctypes import c_void_p

        def up(a):
            a = np.ascontiguousarray(a)
            return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(device)

        self.n_msgs = int(msg_off.shape[0])
        self.n_scope = int(scope.shape[0])
        self.wire_len = int(wire.size)
        self.now = int(now)
        self._t = {"wire": up(wire if wire.size else np.zeros(1, np.uint8)), "off": up(msg_off.astype(np.uint64)),
                   "len": up(msg_len.astype(np.uint32)), "scope": up(scope)}
        self.results = torch.zeros(self.n_msgs * 16 + 16, dtype=torch.uint8, device=device)
        self.winfo = torch.zeros(self.n_msgs * 48 + 48, dtype=torch.uint8, device=device)
        t = self._t
        self.wire_ptr = c_void_p(t["wire"].data_ptr())
        self.off_ptr = c_void_p(t["off"].data_ptr())
        self.len_ptr = c_void_p(t["len"].data_ptr())
        self.scope_ptr = c_void_p(t["scope"].data_ptr())
        self.results_ptr = c_void_p(self.results.data_ptr())
        self.winfo_ptr = c_void_p(self.winfo.data_ptr())

    def results_numpy(self) -> np.ndarray:
        return self.results[: self.n_msgs * 16].cpu().numpy().view(_ffi.RESULT_DTYPE)

    def winfo_numpy(self) -> np.ndarray:
        return self.winfo[: self.n_msgs * 48].cpu().numpy().view(_ffi.WIRE_PROPOSAL_DTYPE)
