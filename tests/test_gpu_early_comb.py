"""HLC_OPT_EARLY_COMB: the device-resident path with the u1 G comb split off the finish (k_rec_ucomb,
enqueued behind the prehash and the prep stage so that it runs in k_rec_main's tail, then k_rec_add
after k_rec_main; the default since round 6).  u1 G goes through memory between the two kernels, so every outcome must be the fused k_rec_comb's: per-vote
statuses, scheme reasons, recovered addresses and per-proposal results on a config-5 Byzantine batch
built on the device, bit for bit against the default context and the C oracle, with and without the
checked chains (HLC_OPT_REC_FORCE_EXACT)."""
import numpy as np
import pytest

import coracle
from hashgraph_like_consensus import byzantine, synth
from hashgraph_like_consensus.device import DeviceBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def early_engine(engine):
    """The default context runs the early comb; `engine` is switched to the fused k_rec_comb for the
    module and back after it, so each test compares the two schedules."""
    from hashgraph_like_consensus.engine import Engine
    eng = Engine(0)
    eng.set_option("early_comb", 1)
    assert eng.get_option("early_comb") == 1
    engine.set_option("early_comb", 0)
    yield eng
    engine.set_option("early_comb", 1)
    eng.close()


def _run(eng, db):
    db.want_recovered()
    eng.validate_proposals_device(db)
    db.torch.cuda.synchronize()
    return (db.results_numpy().copy(), db.status_numpy().copy(), db.reason[: db.n].cpu().numpy().copy(),
            db.recovered[: db.n * 20].cpu().numpy().copy())


@pytest.mark.parametrize("exact", [0, 1])
def test_gpu_early_comb_byzantine_bit_exact(engine, early_engine, exact):
    P, V, start = 400, 64, 123
    seed = synth.config_seed(5)
    db = DeviceBatch.synthetic(engine, P, V, V, True, seed, start_proposal=start)
    kinds = db.make_byzantine(engine, seed, start)
    assert np.array_equal(kinds, byzantine.plan(seed, start, P, V))
    with engine.options(rec_force_exact=exact), early_engine.options(rec_force_exact=exact):
        ref = _run(engine, db)
        got = _run(early_engine, db)
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)
    res, st, rs, _ = got
    vst, vrs, pst, bad, yes, total = byzantine.expectations(kinds, V, db.choice_numpy())
    assert np.array_equal(st, vst) and np.array_equal(res["status"], pst) and np.array_equal(res["bad_index"], bad)
    hb, hd, _ = db.to_host()
    cres, cvst, cvrs, _ = coracle.validate_proposals(hb, hd, db.now, threads=16)
    assert np.array_equal(st, cvst) and np.array_equal(rs, cvrs) and np.array_equal(res, cres)


def test_gpu_early_comb_honest_and_repeated(engine, early_engine):
    """An honest config-2-shaped batch, three calls in a row on the early context (the G rows are
    rewritten per call): every vote valid, results equal to the fused schedule's."""
    db = DeviceBatch.synthetic(engine, 600, 64, 64, True, synth.config_seed(2))
    ref = _run(engine, db)
    assert (ref[1] == 0).all() and (ref[0]["status"] == 0).all()
    for _ in range(3):
        got = _run(early_engine, db)
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)
