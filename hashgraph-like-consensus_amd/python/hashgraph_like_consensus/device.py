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
    def __init__(self, batch: VoteBatch, desc: np.ndarray, now: int, device: str = "cuda:0"):
        import torch
        self.torch = torch

        def up(a):
            a = np.ascontiguousarray(a)
            t = torch.from_numpy(a.view(np.uint8).reshape(-1).copy())
            return t.to(device)

        self.n = batch.n
        self.n_proposals = int(desc.shape[0])
        self.now = int(now)
        arena = batch.arena if batch.arena.size else np.zeros(1, np.uint8)
        self._t = {
            "vote_id": up(batch.vote_id), "proposal_id": up(batch.proposal_id), "timestamp": up(batch.timestamp),
            "vote": up(batch.vote), "bytes": up(arena), "field_off": up(batch.field_off),
            "field_len": up(batch.field_len), "props": up(desc),
        }
        self.results = torch.zeros(self.n_proposals * 16 + 16, dtype=torch.uint8, device=device)
        self.status = torch.zeros(self.n + 1, dtype=torch.uint8, device=device)
        self.reason = torch.zeros(self.n + 1, dtype=torch.uint8, device=device)
        t = self._t
        self.view = _ffi.hlc_votes(
            n=self.n,
            vote_id=ctypes.cast(t["vote_id"].data_ptr(), POINTER(c_uint32)),
            proposal_id=ctypes.cast(t["proposal_id"].data_ptr(), POINTER(c_uint32)),
            timestamp=ctypes.cast(t["timestamp"].data_ptr(), POINTER(c_uint64)),
            vote=ctypes.cast(t["vote"].data_ptr(), POINTER(c_uint8)),
            bytes=ctypes.cast(t["bytes"].data_ptr(), POINTER(c_uint8)),
            bytes_len=int(batch.arena.size),
            field_off=ctypes.cast(t["field_off"].data_ptr(), POINTER(c_uint64)),
            field_len=ctypes.cast(t["field_len"].data_ptr(), POINTER(c_uint32)),
        )
        self.props_ptr = ctypes.cast(t["props"].data_ptr(), POINTER(_ffi.hlc_proposal))
        self.results_ptr = ctypes.cast(self.results.data_ptr(), POINTER(_ffi.hlc_result))
        self.status_ptr = ctypes.cast(self.status.data_ptr(), POINTER(c_uint8))
        self.reason_ptr = ctypes.cast(self.reason.data_ptr(), POINTER(c_uint8))

    def results_numpy(self) -> np.ndarray:
        raw = self.results[: self.n_proposals * 16].cpu().numpy()
        return raw.view(_ffi.RESULT_DTYPE)

    def status_numpy(self) -> np.ndarray:
        return self.status[: self.n].cpu().numpy()


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
