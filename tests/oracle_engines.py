"""Engine doubles whose batch entry points are computed by the oracles (TEST INFRASTRUCTURE):
used by the CPU multi-process tests to check sharding / gathering logic without a GPU."""
from __future__ import annotations

import numpy as np

import coracle
import pyoracle as po
import stream_oracle as so
import wire_oracle as wo
from adversarial import batch_to_votes
from hashgraph_like_consensus import _ffi
from hashgraph_like_consensus.batch import ProposalConfig, pack_proposals


class OracleEngine:
    def validate_proposals(self, batch, desc, now, want_votes=True, want_recovered=False):
        return coracle.validate_proposals(batch, desc, now, threads=2)

    def validate_wire_proposals(self, wire, msg_off, msg_len, scope, now):
        """hlc_validate_wire_proposals semantics: wire_oracle decode + coracle validation."""
        wire = np.asarray(wire, np.uint8)
        m = msg_off.shape[0]
        res = np.zeros(m, _ffi.RESULT_DTYPE)
        winfo = np.zeros(m, _ffi.WIRE_PROPOSAL_DTYPE)
        ok_props, ok_idx, cfgs = [], [], []
        for i in range(m):
            msg = wire[int(msg_off[i]):int(msg_off[i]) + int(msg_len[i])].tobytes()
            code, p, bad = wo.decode_proposal_ex(msg)
            winfo[i]["decode_status"], winfo[i]["bad_vote"] = code, bad
            if code != wo.OK:
                res[i] = (17, 0, code, 0, bad, 0, 0)
                continue
            for k, f in (("name", "name"), ("payload", "payload"), ("owner", "proposal_owner")):
                winfo[i][f"{k}_off"], winfo[i][f"{k}_len"] = getattr(p, f)
            winfo[i]["round"] = p.round
            sl = lambda t: msg[t[0]:t[0] + t[1]]  # noqa: E731
            votes = [po.Vote(vote_id=v.vote_id, vote_owner=sl(v.vote_owner), proposal_id=v.proposal_id,
                             timestamp=v.timestamp, vote=v.vote, parent_hash=sl(v.parent_hash),
                             received_hash=sl(v.received_hash), vote_hash=sl(v.vote_hash),
                             signature=sl(v.signature)) for v in p.votes]
            ok_props.append(po.Proposal(proposal_id=p.proposal_id, votes=votes,
                                        expected_voters_count=p.expected_voters_count, timestamp=p.timestamp,
                                        expiration_timestamp=p.expiration_timestamp,
                                        liveness_criteria_yes=p.liveness_criteria_yes))
            sc = scope[0] if scope.shape[0] == 1 else scope[i]
            cfgs.append(ProposalConfig(float(sc["consensus_threshold"]), int(sc["max_rounds"]),
                                       bool(sc["use_gossipsub_rounds"])))
            ok_idx.append(i)
        if ok_props:
            batch, desc = pack_proposals(ok_props, cfgs)
            r, _, _, _ = coracle.validate_proposals(batch, desc, now, threads=2)
            res[np.array(ok_idx)] = r
        return res, winfo, 0

    def process_votes(self, batch, vote_session, sessions, owners=None, owner_session=None, now=0):
        """hlc_process_votes semantics through oracle/stream_oracle.py (sessions updated in place)."""
        ss = [so.Session(int(x["proposal_id"]), int(x["timestamp"]), int(x["expiration_timestamp"]),
                         int(x["expected_voters_count"]), int(x["round"]), int(x["total"]), int(x["yes"]),
                         int(x["max_rounds"]), float(x["consensus_threshold"]), int(x["state"]),
                         bool(x["use_gossipsub_rounds"]), bool(x["liveness_criteria_yes"])) for x in sessions]
        for o, k in zip(owners if owners is not None else [], owner_session if owner_session is not None else []):
            ss[int(k)].owners.add(bytes(o))
        out = so.process_incoming_votes(ss, batch_to_votes(batch),
                                        [int(v) if v != 0xFFFFFFFF else -1 for v in vote_session], now)
        for k, x in enumerate(ss):
            sessions[k]["round"], sessions[k]["total"], sessions[k]["yes"], sessions[k]["state"] = (
                x.round, x.total, x.yes, x.state)
        cols = list(zip(*out)) if out else [(), (), (), ()]
        return tuple(np.array(c, np.uint8) for c in cols)
