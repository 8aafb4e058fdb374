"""The fixed-base tables (the recovery's u1 G comb and the signing comb) exist once per device per process
(hlc_api.cpp gen_tables): a context created while another lives shares them, the last context destroyed
frees them, and a context created after that builds them again.  Whichever context built them, every
context must recover what the oracle recovers, and closing one must not disturb the others."""
import os
import subprocess
import sys

import pytest

from test_gpu_parity import _mutated_items, _oracle_verify

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpu_tables_shared_between_contexts(engine):
    from hashgraph_like_consensus.engine import Engine
    ids, pays, sigs = _mutated_items(300, 31)
    exp_st, exp_addr = _oracle_verify(ids, pays, sigs)

    def check(e):
        st, addr = e.eth_verify_batch(ids, pays, sigs)
        assert [int(x) for x in st] == exp_st
        assert [a.tobytes() for a in addr] == exp_addr

    a = Engine(0)
    b = Engine(0)
    check(a)
    a.close()        # b and the session's engine still hold the tables
    check(b)
    check(engine)
    b.close()
    check(engine)


CHILD = r"""
import sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {tests!r}); sys.path.insert(0, {oracle!r})
import numpy as np
from hashgraph_like_consensus import synth
from hashgraph_like_consensus.engine import Engine
runs = []
for k in range(3):   # each context is the only one: the tables are built, used and freed three times
    eng = Engine(0)
    w = synth.generate(8, 16, 16, True, 0x484C4361, *synth.engine_signers(eng))
    res, vst, _, _ = eng.validate_proposals(w.batch, w.desc, w.now, want_votes=True)
    assert (vst == 0).all() and (res["status"] == 0).all()
    runs.append((res.tobytes(), vst.tobytes()))
    eng.close()
assert runs[0] == runs[1] == runs[2]
print("child ok", flush=True)
"""


def test_gpu_tables_rebuilt_after_last_context():
    code = CHILD.format(pkg=os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"),
                        tests=os.path.join(ROOT, "tests"), oracle=os.path.join(ROOT, "oracle"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, f"exit {out.returncode}\n{out.stdout[-2000:]}\n{out.stderr[-4000:]}"
    assert "child ok" in out.stdout
