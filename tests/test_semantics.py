"""Validation semantics on the CPU: the reference's behavioural tests (scenarios.py) and a
config-5 adversarial mix, judged identically by the two independent CPU restatements."""
import numpy as np
import pytest

import coracle
import pyoracle as po
from adversarial import byzantine, config_of, proposals_from_batch
from hashgraph_like_consensus.batch import ProposalConfig, pack_proposals
from helpers import oracle_workload
from scenarios import scenarios

SCEN = scenarios()


def pack_scenarios(items):
    props = [p for _, p, _, _, _ in items]
    cfgs = [ProposalConfig(c.consensus_threshold, c.max_rounds, c.use_gossipsub_rounds) for _, _, c, _, _ in items]
    return pack_proposals(props, cfgs)


@pytest.mark.parametrize("name,prop,cfg,now,code", SCEN, ids=[s[0] for s in SCEN])
def test_scenario_python_oracle(name, prop, cfg, now, code):
    assert po.from_proposal(prop, cfg, now).status == code


def test_scenarios_c_oracle_matches_python():
    # one batch per distinct `now` (the ABI takes one now per call)
    for now in sorted({s[3] for s in SCEN}):
        items = [s for s in SCEN if s[3] == now]
        batch, desc = pack_scenarios(items)
        res, vst, vrs, rec = coracle.validate_proposals(batch, desc, now, threads=2)
        for k, (name, p, cfg, _, code) in enumerate(items):
            out = po.from_proposal(p, cfg, now)
            assert int(res[k]["status"]) == out.status == code, name
            assert int(res[k]["transition"]) == out.transition, name
            if out.status == po.OK:
                assert (int(res[k]["yes"]), int(res[k]["total"])) == (out.yes, out.total), name
            else:
                bi = int(res[k]["bad_index"])
                assert (bi if bi != 0xFFFFFFFF else -1) == out.bad_index, name


def test_transitions_of_scenarios():
    by = {s[0]: s for s in SCEN}
    o = po.from_proposal(by["p2p_batch_6_of_9"][1], by["p2p_batch_6_of_9"][2], by["p2p_batch_6_of_9"][3])
    assert o.transition == po.REACHED_YES and o.round == 7
    o = po.from_proposal(by["gossipsub_batch_3_of_5"][1], po.ConsensusConfig.gossipsub(), by["gossipsub_batch_3_of_5"][3])
    assert o.transition == po.STILL_ACTIVE and o.round == 2   # 3 < ceil(10/3) = 4
    o = po.from_proposal(by["single_voter_no"][1], po.ConsensusConfig.gossipsub(), by["single_voter_no"][3])
    assert o.transition == po.REACHED_NO
    o = po.from_proposal(by["tie_liveness_false"][1], po.ConsensusConfig.gossipsub(), by["tie_liveness_false"][3])
    assert o.transition == po.REACHED_NO


def test_adversarial_mix_python_vs_c():
    w = oracle_workload(10, 12, 12, True, 0x484C4305)
    batch, desc, kinds = byzantine(w, fraction=1 / 3, seed=11)
    res, vst, vrs, rec = coracle.validate_proposals(batch, desc, w.now, threads=4)
    props = proposals_from_batch(batch, desc)
    seen = set()
    for k, p in enumerate(props):
        out = po.from_proposal(p, config_of(desc[k]), w.now)
        assert int(res[k]["status"]) == out.status
        bi = int(res[k]["bad_index"])
        assert (bi if bi != 0xFFFFFFFF else -1) == out.bad_index
        seen.add(out.status)
    # per-vote statuses against the Python restatement
    b = 0
    for k, p in enumerate(props):
        for j, v in enumerate(p.votes):
            st, rs = po.vote_status_in_proposal(p, v, w.now)
            assert (int(vst[b + j]), int(vrs[b + j])) == (st, rs)
        b += len(p.votes)
    assert len(seen) >= 4


def test_c_oracle_reverify_never_fails():
    w = oracle_workload(4, 16, 16, True, 9)
    coracle.validate_proposals(w.batch, w.desc, w.now, threads=2, reverify=True)
    assert coracle.verify_failures() == 0
