"""Process teardown with libhlc contexts the caller never closed (a SIGSEGV inside
__cxa_finalize after a host-pipeline tool had written its outputs).  _ffi's atexit hook destroys every
live context -- streams, events, device and page-locked buffers, the parked threads of the host staging
pool -- before the library finalizers run.  Each case is one fresh child process, started once; its exit
status must be 0."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {tests!r}); sys.path.insert(0, {oracle!r})
import numpy as np
from hashgraph_like_consensus import _ffi, synth
from hashgraph_like_consensus.engine import Engine
eng = Engine(0)
w = synth.generate(4, 8, 8, True, 0x484C4361, *synth.engine_signers(eng))
res, vst, _, _ = eng.validate_proposals(w.batch, w.desc, w.now, want_votes=True)
assert (vst == 0).all() and (res["status"] == 0).all()
wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
wres, _, _ = eng.validate_wire_proposals(wire, off, lens, scope, w.now)
assert np.array_equal(wres, res)
st, _ = eng.eth_verify_batch([b"\x00" * 20], [b"x"], [b"\x00" * 65])
{extra}
print("child ok", flush=True)
"""


@pytest.mark.parametrize("extra", [
    "",                                                     # never closed: the atexit hook destroys it
    "pb = w.batch.pinned(); eng.validate_proposals(pb, w.desc, w.now)",  # a live page-locked arena too
    "eng2 = Engine(0); eng2.validate_proposals(w.batch, w.desc, w.now)",  # two contexts left open
    "eng.close()",                                          # closed by the caller (the hook skips it)
])
def test_gpu_exit_without_close(extra):
    code = CHILD.format(pkg=os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"),
                        tests=os.path.join(ROOT, "tests"), oracle=os.path.join(ROOT, "oracle"), extra=extra)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, f"exit {out.returncode}\n{out.stdout[-2000:]}\n{out.stderr[-4000:]}"
    assert "child ok" in out.stdout
