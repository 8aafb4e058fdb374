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


def test_gpu_early_comb_host_entries(early_engine):
    """Bit 2 of HLC_OPT_EARLY_COMB: the host-buffer entries' finish with k_rec_ucomb behind every
    recovery range's prep stage (records at the call's row stride) equals the fused finish, for the
    SoA entry over several recovery ranges and the pipelined wire entry over several message ranges;
    the SoA outcomes also equal the C oracle's."""
    from adversarial import byzantine as byz_mix
    from helpers import oracle_workload
    w = oracle_workload(260, 64, 64, True, 0xEC0B)
    batch, desc, _ = byz_mix(w, fraction=1 / 3, seed=0xEC0B)
    outs = {}
    for mode in (0, 3):
        with early_engine.options(early_comb=mode, split_votes=[2048, 4096]):
            outs[mode] = early_engine.validate_proposals(batch, desc, w.now, want_recovered=True)
    for a, b in zip(outs[0], outs[3]):
        assert np.array_equal(a, b)
    cres, cvst, cvrs, crec = coracle.validate_proposals(batch, desc, w.now)
    res, vst, vrs, rec = outs[3]
    assert np.array_equal(vst, cvst) and np.array_equal(vrs, cvrs) and np.array_equal(rec, crec)
    assert np.array_equal(res, cres)
    wire, off, lens, scope = synth.to_wire(batch, desc)
    wouts = {}
    for mode in (0, 3):
        with early_engine.options(early_comb=mode, wire_split_bytes=[8192, 16384], wire_chunk=4096, host_trace=2):
            wouts[mode] = early_engine.validate_wire_proposals(wire, off, lens, scope, w.now)
            assert early_engine.last_host_trace()["facts"]["ranges"] >= 2
    assert wouts[0][2] == wouts[3][2]
    assert np.array_equal(wouts[0][0], wouts[3][0])
    assert np.array_equal(wouts[0][1].view(np.uint8), wouts[3][1].view(np.uint8))
