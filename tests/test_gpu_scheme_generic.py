"""GPU parity of the scheme-generic boundary: `ConsensusService<.., Signer>` for a Signer other than
EthereumConsensusSigner (/root/reference/src/service.rs:39-51, src/signing.rs:46-74), through
hlc_validate_proposals_verdicts[_device], hlc_process_votes_verdicts and hlc_encode_vote_payloads.

  * the reference's own custom-scheme tests restated on the product service with its StubSigner
    (tests/custom_scheme_tests.rs:91-136: three stub voters reach consensus; :139-178: a forged
    signature is InvalidVoteSignature), at the proposal level and the incoming-vote level;
  * a Byzantine stub-scheme mix (forged and short signatures, wrong-length identities -> Err(Verify),
    tampered hashes, empty fields, timestamps, pid, broken links, duplicates) bit-exact against the C
    oracle's stub scheme (HLCO_STUB) and pyoracle, per vote and per proposal, host and device entries;
  * the device payload encoder equals the prost encoding of both oracles;
  * hlc_eth_verify_batch's statuses fed back as verdicts reproduce hlc_validate_proposals bit for bit
    on a config-5 Ethereum mix (the verdict entry adds nothing and loses nothing);
  * the streaming path under the stub scheme equals oracle/stream_oracle.py with stub_verify.
"""
import copy
import random

import numpy as np
import pytest

import coracle
import pyoracle as po
import stream_oracle as so
from adversarial import byzantine
from hashgraph_like_consensus import _ffi, errors
from hashgraph_like_consensus.protos import Proposal, Vote
from hashgraph_like_consensus.service import ConsensusConfig, ConsensusService, build_vote
from hashgraph_like_consensus.signing import scheme_verdicts
from helpers import oracle_workload
from stream_cases import sessions_array
from stub_scheme import NOW, StubSigner, stub_workload

pytestmark = pytest.mark.gpu


def _compare(engine, batch, desc, now, label):
    verdicts = scheme_verdicts(StubSigner, batch, engine)
    res, vst, vrs = engine.validate_proposals_verdicts(batch, desc, now, verdicts)
    cres, cvst, cvrs, _ = coracle.validate_proposals(batch, desc, now, threads=8, scheme="stub")
    bad = np.nonzero((vst != cvst) | (vrs != cvrs))[0]
    assert bad.size == 0, f"{label}: {bad.size} votes differ, first {bad[:5]} gpu {vst[bad[:5]]} cpu {cvst[bad[:5]]}"
    badp = np.nonzero(res != cres)[0]
    assert badp.size == 0, f"{label}: {badp.size} proposals differ, first {badp[:5]}"
    return res, vst, vrs, verdicts


@pytest.mark.parametrize("seed", [3, 4])
def test_gpu_stub_byzantine_mix_bit_exact(engine, seed):
    props, batch, desc, now, kinds = stub_workload(120, 16, seed, fraction=0.35)
    res, vst, vrs, _ = _compare(engine, batch, desc, now, "mix")
    assert {po.OK, po.SIGNATURE_SCHEME, po.INVALID_VOTE_SIGNATURE, po.INVALID_VOTE_HASH} <= set(res["status"].tolist())
    assert (vrs[vst == po.SIGNATURE_SCHEME] == po.SCHEME_PLUGIN).all()
    props, batch, desc, now, kinds = stub_workload(90, 12, seed + 20, fraction=0.1,
                                                   kinds_pool=["bad_received", "duplicate"])
    res, _, _, _ = _compare(engine, batch, desc, now, "chain/dup")
    assert {po.OK, po.DUPLICATE_VOTE, po.RECEIVED_HASH_MISMATCH} <= set(res["status"].tolist())


def test_gpu_stub_larger_batch_and_device_entry(engine):
    """~20k stub-scheme votes (one proposal of 600 votes takes the global-table chain path), host entry
    vs C oracle, then the device entry on the same batch equals the host entry."""
    import torch
    from hashgraph_like_consensus.device import DeviceBatch
    props, batch, desc, now, kinds = stub_workload(300, 64, 11, fraction=0.05, clean_every=2)
    big, bb, bd, _, _ = stub_workload(1, 600, 12, fraction=0.0)
    from stub_scheme import pack
    batch, desc = pack(props + big)
    res, vst, vrs, verdicts = _compare(engine, batch, desc, now, "20k")
    assert int((res["status"] == 0).sum()) >= 150 and int(res[-1]["status"]) == 0 and int(res[-1]["total"]) == 600
    db = DeviceBatch(batch, desc, now)
    dv = torch.from_numpy(verdicts.copy()).to("cuda:0")
    torch.cuda.synchronize()
    engine.validate_proposals_verdicts_device(db, dv.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(db.results_numpy(), res)
    assert np.array_equal(db.status_numpy(), vst)
    assert np.array_equal(db.reason[: db.n].cpu().numpy(), vrs)


def test_gpu_encode_payloads_match_oracles(engine):
    props, batch, desc, now, _ = stub_workload(20, 8, 5, fraction=0.4)
    arena, off, lens = engine.encode_vote_payloads(batch)
    votes = [v for p in props for v in p.votes]
    for i, v in enumerate(votes):
        got = arena[int(off[i]):int(off[i]) + int(lens[i])].tobytes()
        assert got == po.signed_payload(v), i
    # Ethereum batch, incl. proto3 defaults (vote_id 0, timestamp 0, vote false, empty fields)
    w = oracle_workload(4, 8, 8, True, 0x484C4371)
    b = w.batch
    b.vote_id[3] = 0
    b.timestamp[5] = 0
    b.vote[:] = 0
    b.field_len[7, :] = 0
    arena, off, lens = engine.encode_vote_payloads(b)
    for i in range(b.n):
        assert arena[int(off[i]):int(off[i]) + int(lens[i])].tobytes() == coracle.encode_vote(b, i), i


def test_gpu_eth_verdicts_reproduce_validate_proposals(engine):
    """Config-5 Ethereum mix: hlc_eth_verify_batch over (owner, payload, signature) of every vote, fed as
    verdicts, gives exactly hlc_validate_proposals' statuses, scheme reasons and proposal results."""
    w = oracle_workload(40, 16, 16, True, 0x484C4372)
    bbatch, desc, _ = byzantine(w, fraction=1 / 3, seed=7)
    res, vst, vrs, _ = engine.validate_proposals(bbatch, desc, w.now)
    arena, off, lens = engine.encode_vote_payloads(bbatch)
    n = bbatch.n
    items = [(bbatch.field(i, 0), arena[int(off[i]):int(off[i]) + int(lens[i])].tobytes(), bbatch.field(i, 4))
             for i in range(n)]
    st, _ = engine.eth_verify_batch([a for a, _, _ in items], [p for _, p, _ in items], [s for _, _, s in items])
    res2, vst2, vrs2 = engine.validate_proposals_verdicts(bbatch, desc, w.now, st)
    assert np.array_equal(vst2, vst) and np.array_equal(vrs2, vrs) and np.array_equal(res2, res)
    assert len(set(vrs.tolist())) >= 4


def test_gpu_verdicts_reject_bad_codes(engine):
    props, batch, desc, now, _ = stub_workload(2, 4, 6)
    bad = np.zeros(batch.n, np.uint8)
    bad[3] = _ffi.VERIFY_ERR + 1
    with pytest.raises(_ffi.HlcError):
        engine.validate_proposals_verdicts(batch, desc, now, bad)
    with pytest.raises(ValueError):
        engine.validate_proposals_verdicts(batch, desc, now, bad[:-1])


def _stub_vote(proposal: Proposal, signer: StubSigner, now: int, engine, choice=True) -> Vote:
    return build_vote(proposal, choice, signer, now, engine)


def test_gpu_reference_custom_scheme_reaches_consensus(engine):
    """custom_scheme_tests.rs:91-136 on the product service: three StubSigner peers vote YES on a
    Gossipsub proposal of 3 expected voters -> ConsensusReached(true), through the incoming-vote path
    (hlc_process_votes_verdicts) and through one incoming proposal carrying the votes."""
    now = NOW
    owner, two, three = StubSigner(bytes([1] * 8)), StubSigner(bytes([2] * 8)), StubSigner(bytes([3] * 8))
    svc = ConsensusService(engine, ConsensusConfig.gossipsub(), scheme=StubSigner)
    p = Proposal(name="stub-proposal", payload=b"payload", proposal_id=4242, proposal_owner=owner.identity(),
                 expected_voters_count=3, timestamp=now, expiration_timestamp=now + 60, liveness_criteria_yes=True)
    svc.process_incoming_proposal("stub-scope", copy.deepcopy(p), now)
    carrier = copy.deepcopy(p)
    for signer in (owner, two, three):
        v = _stub_vote(carrier, signer, now, engine)
        carrier.votes.append(v)
        svc.process_incoming_vote("stub-scope", v, now)
    rec = svc.get_session("stub-scope", 4242)
    # the reference's assertion (custom_scheme_tests.rs:130-135): consensus reached, YES.  Two YES votes of
    # three already decide it (ceil(2n/3) = 2); the third is then accepted without entering the map, as
    # add_vote does on a decided session (session.rs:247)
    assert rec.consensus is True and (rec.total, rec.yes) == (2, 2)
    # the same votes inside one incoming proposal (another scope): from_proposal reaches consensus
    svc2 = ConsensusService(engine, ConsensusConfig.gossipsub(), scheme=StubSigner)
    o = svc2.process_incoming_proposals("stub-scope-2", [carrier], now)[0]
    assert o.ok and o.consensus is True and (o.yes, o.total) == (3, 3)
    # the Ethereum service rejects the same proposal: 8-byte identities are not addresses
    o_eth = ConsensusService(engine).process_incoming_proposals("eth", [copy.deepcopy(carrier)], now)[0]
    assert isinstance(o_eth.error, errors.SignatureScheme)


def test_gpu_reference_custom_scheme_rejects_forged_signature(engine):
    """custom_scheme_tests.rs:139-178: a vote whose signature bytes are all flipped is rejected with
    InvalidVoteSignature by process_incoming_vote."""
    now = NOW
    owner, voter = StubSigner(bytes([9] * 8)), StubSigner(bytes([10] * 8))
    svc = ConsensusService(engine, ConsensusConfig.gossipsub(), scheme=StubSigner)
    p = Proposal(name="stub-proposal", payload=b"payload", proposal_id=99, proposal_owner=owner.identity(),
                 expected_voters_count=2, timestamp=now, expiration_timestamp=now + 60, liveness_criteria_yes=True)
    svc.process_incoming_proposal("stub-scope-forge", copy.deepcopy(p), now)
    v = _stub_vote(p, voter, now, engine)
    v.signature = bytes(b ^ 0xFF for b in v.signature)
    with pytest.raises(errors.InvalidVoteSignature):
        svc.process_incoming_vote("stub-scope-forge", v, now)
    # an identity of the wrong length is the stub's Err(Verify) -> SignatureScheme
    w = _stub_vote(p, voter, now, engine)
    w.vote_owner = bytes([10] * 7)
    w.vote_hash = b""
    from hashgraph_like_consensus.service import compute_vote_hash
    from hashgraph_like_consensus.protos import encode_vote
    w.signature = b""
    w.vote_hash = compute_vote_hash(w, engine)
    w.signature = StubSigner.expected_signature(w.vote_owner, encode_vote(w))
    with pytest.raises(errors.SignatureScheme):
        svc.process_incoming_vote("stub-scope-forge", w, now)


def test_gpu_stub_streaming_matches_oracle(engine):
    """process_incoming_vote micro-batches under the stub scheme: shuffled deliveries with replays,
    Byzantine votes and storage misses across sessions that already hold owners of several lengths."""
    rnd = random.Random(77)
    props, batch, desc, now, kinds = stub_workload(24, 10, 21, fraction=0.3)
    sessions, deliveries = [], []
    for k, p in enumerate(props):
        s = so.Session(proposal_id=p.proposal_id, timestamp=p.timestamp, expiration_timestamp=p.expiration_timestamp,
                       expected_voters_count=p.expected_voters_count + rnd.choice([0, 2]), round=1, total=0, yes=0,
                       max_rounds=2, consensus_threshold=2.0 / 3.0, state=po.SESSION_ACTIVE, use_gossipsub_rounds=True,
                       liveness_criteria_yes=True)
        pre = rnd.choice([0, 1, 2])
        for j in range(pre):  # owners already in the map (one of them a 20-byte identity)
            s.owners.add(p.votes[j].vote_owner if j == 0 else bytes([k, j] * 10))
            s.total += 1
            s.round = 2
        sessions.append(s)
        for v in p.votes[pre:]:
            deliveries.append((v, k))
            if rnd.random() < 0.15:
                deliveries.append((v, k))
    rnd.shuffle(deliveries)
    deliveries.insert(3, (deliveries[0][0], -1))
    votes = [v for v, _ in deliveries]
    vs = [k for _, k in deliveries]
    ss_ref = copy.deepcopy(sessions)
    out_ref = so.process_incoming_votes(ss_ref, votes, vs, now, po.stub_verify)
    from hashgraph_like_consensus.batch import pack_votes
    vb = pack_votes(votes)
    verdicts = scheme_verdicts(StubSigner, vb, engine)
    orows, osess = [], []
    for k, s in enumerate(sessions):
        for o in sorted(s.owners):
            orows.append(o)
            osess.append(k)
    sarr = sessions_array(sessions)
    vsess = np.array([0xFFFFFFFF if k < 0 else k for k in vs], np.uint32)
    st, tr, ins, rs = engine.process_votes_verdicts(vb, vsess, sarr, orows, np.array(osess, np.uint32), now, verdicts)
    exp = np.array([(o[0], o[1], int(o[2]), o[3]) for o in out_ref], np.int64)
    got = np.stack([st, tr, ins, rs], axis=1).astype(np.int64)
    bad = np.nonzero((exp != got).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} votes differ, first {bad[:5]}: gpu {got[bad[:3]]} ref {exp[bad[:3]]}"
    assert np.array_equal(sarr, sessions_array(ss_ref))
    codes = {o[0] for o in out_ref}
    assert {po.OK, po.DUPLICATE_VOTE, po.SIGNATURE_SCHEME, po.INVALID_VOTE_SIGNATURE, 19} <= codes


def test_gpu_stub_proposal_bytes_matches_oracle(engine):
    """Gossip bytes under the stub scheme: ConsensusService(scheme=StubSigner).process_incoming_proposal_bytes
    decodes on the device and validates with the scheme's verdicts; every outcome equals pyoracle's
    from_proposal under stub_verify."""
    from hashgraph_like_consensus.protos import encode_proposal
    props, batch, desc, now, kinds = stub_workload(30, 6, 31, fraction=0.3)
    msgs = []
    for p in props:
        pp = Proposal(name=p.name, payload=p.payload, proposal_id=p.proposal_id, proposal_owner=p.proposal_owner,
                      votes=[Vote(**v.__dict__) for v in p.votes], expected_voters_count=p.expected_voters_count,
                      round=1, timestamp=p.timestamp, expiration_timestamp=p.expiration_timestamp,
                      liveness_criteria_yes=p.liveness_criteria_yes)
        msgs.append(encode_proposal(pp))
    svc = ConsensusService(engine, ConsensusConfig.gossipsub(), scheme=StubSigner)
    outs = svc.process_incoming_proposal_bytes("stub-wire", msgs, now)
    cfg = po.ConsensusConfig.gossipsub()
    for p, o in zip(props, outs):
        ref = po.from_proposal(p, cfg, now, scheme=po.stub_verify)
        got = 0 if o.error is None else o.error.code
        assert got == ref.status, (p.proposal_id, got, ref.status)
        assert o.bad_index == ref.bad_index
        if ref.status == po.OK:
            assert (o.yes, o.total) == (ref.yes, ref.total)
    assert len({0 if o.error is None else o.error.code for o in outs}) >= 3


def test_gpu_stub_long_fields_take_the_general_path(engine):
    """Votes whose SHA-256 input outgrows the fused kernel's LDS window (k_prehash_fused defers them to the
    streaming k_prehash_stream) under the stub scheme: 300-byte parent hashes and identities, re-hashed and
    re-signed, beside ordinary votes -- every status, reason and proposal outcome equals the C oracle's."""
    import hashlib
    from stub_scheme import _finish, pack
    rnd = random.Random(91)
    props, _, _, now, _ = stub_workload(24, 6, 41)
    for p in props:
        for j, v in enumerate(p.votes):
            r = rnd.random()
            if r < 0.25:
                v.parent_hash = hashlib.sha256(bytes([j])).digest() * 10  # 320 bytes: no such vote
            elif r < 0.4:
                v.vote_owner = bytes(rnd.getrandbits(8) for _ in range(300))  # the stub's Err: not 8 bytes
            else:
                continue
            _finish(v)
            if j + 1 < len(p.votes):  # keep the next vote's received link to this one
                nxt = p.votes[j + 1]
                nxt.received_hash = v.vote_hash
                _finish(nxt)
    batch, desc = pack(props)
    res, vst, vrs, _ = _compare(engine, batch, desc, now, "long fields")
    codes = set(res["status"].tolist())
    assert po.SIGNATURE_SCHEME in codes and po.PARENT_HASH_MISMATCH in codes, codes
