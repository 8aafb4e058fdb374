"""GPU: the k_rec_main clock stamps (hlc_ctx_set_clock_probe / hlc_ctx_clock_probe, the bench line's
live_k_rec_main_clock).  Stamped calls give the same outcomes bit for bit as unstamped ones, every wave of
the grid stamps, and the clock is a plausible MI355X shader clock; without a stamped launch the query fails
with HLC_EINVAL."""
import numpy as np
import pytest
import torch

from hashgraph_like_consensus import _ffi, synth

pytestmark = pytest.mark.gpu


def test_gpu_clock_probe_outcomes_and_range(engine):
    from hashgraph_like_consensus.device import DeviceBatch
    with pytest.raises(_ffi.HlcError):
        engine.clock_probe()  # nothing stamped yet on this context's setting
    db = DeviceBatch.synthetic(engine, 2_000, 64, 64, True, synth.config_seed(2))
    engine.validate_proposals_device(db)
    torch.cuda.synchronize()
    ref_res, ref_st = db.results_numpy().copy(), db.status_numpy().copy()
    engine.set_clock_probe(True)
    try:
        engine.validate_proposals_device(db)
        torch.cuda.synchronize()
        c = engine.clock_probe()
    finally:
        engine.set_clock_probe(False)
    assert np.array_equal(db.results_numpy().view(np.uint8), ref_res.view(np.uint8))
    assert np.array_equal(db.status_numpy(), ref_st)
    # 128k votes -> 2,000 grabs of 64: every wave of the grid (up to 2,048) has work or exits at once
    assert c["waves"] > 0
    assert 0.8 < c["min_GHz"] <= c["median_GHz"] <= c["max_GHz"] < 2.6, c
