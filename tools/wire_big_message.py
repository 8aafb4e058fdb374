#!/usr/bin/env python3
"""Decode time of one huge Proposal message (1M vote records) on the device: messages over 1 MiB
take the parallel boundary-discovery path (next[] per byte offset + pointer jumping)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))

from hashgraph_like_consensus import _ffi  # noqa: E402
from hashgraph_like_consensus.engine import Engine  # noqa: E402
from hashgraph_like_consensus.protos import Proposal, Vote, encode_proposal  # noqa: E402


def main() -> None:
    n = 1_000_000
    one = Vote(vote_id=7, vote_owner=b"\x11" * 20, proposal_id=9, timestamp=1_760_000_001, vote=True,
               received_hash=b"\x22" * 32, vote_hash=b"\x33" * 32, signature=b"\x44" * 65)
    msg = encode_proposal(Proposal(name="big", proposal_id=9, votes=[one] * n, expected_voters_count=n,
                                   timestamp=5, expiration_timestamp=9))
    print("encoded", len(msg), flush=True)
    eng = Engine(0)
    sc = np.zeros(1, _ffi.SCOPE_CONFIG_DTYPE)
    wire = np.frombuffer(msg, np.uint8)
    off, ln = np.zeros(1, np.uint64), np.array([len(msg)], np.uint32)
    eng.decode_proposals(wire, off, ln, sc)  # warm-up (allocations)
    print("warm-up done", flush=True)
    t0 = time.perf_counter()
    props, winfo, batch = eng.decode_proposals(wire, off, ln, sc)
    dt = time.perf_counter() - t0
    assert int(winfo[0]["decode_status"]) == 0 and int(props[0]["vote_count"]) == n
    print(json.dumps({"records": n, "message_bytes": len(msg), "decode_call_ms_incl_pcie": dt * 1e3}))


if __name__ == "__main__":
    main()
