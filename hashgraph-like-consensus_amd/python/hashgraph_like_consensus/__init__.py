"""MI355X-native batch vote-validation engine for hashgraph-like-consensus.

Python mirror of the reference crate's public surface for the validation hot path
(/root/reference/src/{utils,signing,session,service}.rs), backed by libhlc.so (HIP, gfx950).
"""
from . import _ffi
from .protos import Proposal, Vote

__all__ = ["Proposal", "Vote", "_ffi"]
__version__ = "0.1.0"
