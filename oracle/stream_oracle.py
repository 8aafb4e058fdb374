"""CPU restatement of `ConsensusService::process_incoming_vote` over a sequence of incoming votes
(TEST INFRASTRUCTURE -- only tests/ may use it, as the checker of hlc_process_votes).

Follows /root/reference/src/service.rs:286-305 per vote, in delivery order:
  get_session (storage lookup: SessionNotFound)                      service.rs:292
  validate_vote(vote, session.expiration, session.timestamp, now)    service.rs:293-298, utils.rs:127-171
  update_session -> ConsensusSession::add_vote(vote, now)             service.rs:300-302, session.rs:225-249
      ConsensusReached(r)  -> Ok(ConsensusReached(r)), vote not inserted
      Failed               -> Err(SessionNotActive)
      Active: validate_proposal_timestamp (now >= exp: ProposalExpired)   utils.rs:320-328
              check_round_limit(1) (may set Failed)                       session.rs:306-344
              owner already in the map -> DuplicateVote                    session.rs:236-238
              insert; update_round(1); check_consensus                     session.rs:239-244, 350-387
The in-memory storage mutates the session in place (storage.rs:301-318), so a Failed state set
by check_round_limit persists even though the call returns an error.

Per-vote validation reuses pyoracle.validate_vote (the restatement pinned by the published KATs).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Set, Tuple

import pyoracle as po

SESSION_NOT_ACTIVE = 18   # error.rs:54
SESSION_NOT_FOUND = 19    # error.rs:56
_U32 = 0xFFFFFFFF


@dataclass
class Session:
    """The fields of hlc_session (include/hlc.h) plus the owner set of the vote map."""
    proposal_id: int
    timestamp: int
    expiration_timestamp: int
    expected_voters_count: int
    round: int
    total: int
    yes: int
    max_rounds: int
    consensus_threshold: float
    state: int
    use_gossipsub_rounds: bool
    liveness_criteria_yes: bool
    owners: Set[bytes] = field(default_factory=set)

    def config(self) -> po.ConsensusConfig:
        return po.ConsensusConfig(self.consensus_threshold, self.max_rounds, self.use_gossipsub_rounds,
                                  self.liveness_criteria_yes)


def _check_round_limit(s: Session, vote_count: int) -> bool:
    """session.rs:306-344; sets Failed when the limit is exceeded."""
    if not po.check_round_limit(s.config(), s.expected_voters_count, s.round, vote_count):
        s.state = po.SESSION_FAILED
        return False
    return True


def _update_round(s: Session, vote_count: int) -> None:
    """session.rs:350-366 (saturating at u32::MAX for P2P)."""
    s.round = po.update_round(s.config(), s.round, vote_count)


def add_vote(s: Session, v: po.Vote, now: int) -> Tuple[int, int, bool]:
    """session.rs:225-249 -> (status, transition, inserted)."""
    if s.state in (po.SESSION_REACHED_NO, po.SESSION_REACHED_YES):
        return po.OK, (po.REACHED_YES if s.state == po.SESSION_REACHED_YES else po.REACHED_NO), False
    if s.state != po.SESSION_ACTIVE:
        return SESSION_NOT_ACTIVE, po.STILL_ACTIVE, False
    if now >= s.expiration_timestamp:
        return po.PROPOSAL_EXPIRED, po.STILL_ACTIVE, False
    if not _check_round_limit(s, 1):
        return po.MAX_ROUNDS_EXCEEDED, po.STILL_ACTIVE, False
    if v.vote_owner in s.owners:
        return po.DUPLICATE_VOTE, po.STILL_ACTIVE, False
    s.owners.add(v.vote_owner)
    s.total += 1
    s.yes += 1 if v.vote else 0
    _update_round(s, 1)
    r = po.calculate_consensus_result(s.total, s.yes, s.expected_voters_count, s.consensus_threshold,
                                      s.liveness_criteria_yes, False)   # check_consensus, session.rs:372-387
    if r is None:
        s.state = po.SESSION_ACTIVE
        return po.OK, po.STILL_ACTIVE, True
    s.state = po.SESSION_REACHED_YES if r else po.SESSION_REACHED_NO
    return po.OK, (po.REACHED_YES if r else po.REACHED_NO), True


def _as_proposal(s: Session) -> po.Proposal:
    return po.Proposal(proposal_id=s.proposal_id, timestamp=s.timestamp, expiration_timestamp=s.expiration_timestamp)


def process_incoming_votes(sessions: List[Session], votes: Sequence[po.Vote], vote_session: Sequence[int],
                           now: int, scheme=po.ethereum_verify) -> List[Tuple[int, int, bool, int]]:
    """service.rs:286-305 for each vote in order -> [(status, transition, inserted, scheme reason)].
    vote_session[i] = session index or -1 / 0xFFFFFFFF for "not found".  Mutates `sessions`.
    `scheme` is the service's `Signer::verify` (pyoracle.ethereum_verify or pyoracle.stub_verify)."""
    out = []
    for v, si in zip(votes, vote_session):
        if si < 0 or si >= len(sessions):
            out.append((SESSION_NOT_FOUND, po.STILL_ACTIVE, False, 0))
            continue
        s = sessions[si]
        # the reference's storage lookup is keyed by vote.proposal_id, so a session of another
        # proposal can only come from a caller's mapping error: reported as the id mismatch
        st, sub = po.vote_status_in_proposal(_as_proposal(s), v, now, scheme)
        if st != po.OK:
            out.append((st, po.STILL_ACTIVE, False, sub))
            continue
        st, tr, ins = add_vote(s, v, now)
        out.append((st, tr, ins, 0))
    return out
