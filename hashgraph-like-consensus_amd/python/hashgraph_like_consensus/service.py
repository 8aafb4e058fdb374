"""Host-side mirror of the reference's entry points onto the hot path.

* `ConsensusConfig`         session.rs:25-160 (gossipsub()/p2p() presets, validated builders)
* `validate_proposal(s)`    utils.rs:106-225 (`validate_proposal`, `validate_vote_chain`, `validate_vote`)
* `compute_vote_hash(es)`   utils.rs:37-52
* `build_vote`              utils.rs:55-104
* `ConsensusService.process_incoming_proposal(s)`  service.rs:263-279 -> session.rs:198-300
* `ConsensusService.handle_consensus_timeout(s)`   service.rs:323-373 (batched tally)
* `ConsensusService.process_incoming_vote(s)`       service.rs:286-305 (micro-batched)
* `ConsensusService.process_incoming_proposal_bytes` wire bytes -> device decode -> service.rs:263-279

Only the slice of `ConsensusService` that sits on the validation path is mirrored: the
duplicate-session check (`ProposalAlreadyExist`), config resolution (service.rs:444-484) and
`ConsensusSession::from_proposal`.  The event bus, storage trait, scope management and timeout
handling are the reference's control plane and are out of scope (DESIGN.md §Out of scope); the
accepted sessions are kept in a plain dict so a second delivery of the same proposal id is
rejected exactly as the reference's storage lookup does.

Every hash, signature and tally is computed on the GPU through libhlc.so (engine.py); this module
only marshals and maps status codes to exceptions.  The service is generic over the signature scheme
like the reference's `ConsensusService<.., Signer>` (service.rs:39-51): with the default
EthereumConsensusSigner the device runs the whole validation; with any other
`ConsensusSignatureScheme` (e.g. the reference's StubSigner, tests/custom_scheme_tests.rs) the scheme's
`verify_batch` decides the signature step of each vote and the device runs everything else
(hlc_validate_proposals_verdicts / hlc_process_votes_verdicts).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import errors
from .batch import ProposalConfig, pack_proposals, pack_votes
from .engine import Engine
from .protos import Proposal, Vote
from .signing import scheme_verdicts

GOSSIPSUB, P2P = "gossipsub", "p2p"
DEFAULT_THRESHOLD = 2.0 / 3.0
DEFAULT_TIMEOUT_S = 60

TRANSITION_STILL_ACTIVE, TRANSITION_CONSENSUS_REACHED = 0, 1


@dataclass(frozen=True)
class ConsensusConfig:
    """session.rs:25-44.  Defaults are `ConsensusConfig::gossipsub()` (scope_config.rs defaults:
    threshold 2/3, timeout 60 s, max_rounds 2, liveness_criteria_yes true)."""
    consensus_threshold: float = DEFAULT_THRESHOLD
    consensus_timeout: int = DEFAULT_TIMEOUT_S
    max_rounds: int = 2
    use_gossipsub_rounds: bool = True
    liveness_criteria: bool = True

    @staticmethod
    def gossipsub() -> "ConsensusConfig":
        return ConsensusConfig()

    @staticmethod
    def p2p() -> "ConsensusConfig":
        """max_rounds 0 = derive ceil(2n/3)-style cap from expected_voters_count (session.rs:120-128)."""
        return ConsensusConfig(max_rounds=0, use_gossipsub_rounds=False)

    def with_threshold(self, t: float) -> "ConsensusConfig":
        if not (0.0 <= t <= 1.0):          # utils.rs:331-336
            raise errors.InvalidConsensusThreshold()
        return dataclasses.replace(self, consensus_threshold=float(t))

    def with_timeout(self, seconds: int) -> "ConsensusConfig":
        if seconds <= 0:                    # utils.rs:339-344
            raise errors.InvalidTimeout()
        return dataclasses.replace(self, consensus_timeout=int(seconds))

    def with_liveness_criteria(self, yes: bool) -> "ConsensusConfig":
        return dataclasses.replace(self, liveness_criteria=bool(yes))

    def with_max_rounds(self, max_rounds: int) -> "ConsensusConfig":
        return dataclasses.replace(self, max_rounds=int(max_rounds))

    def to_proposal_config(self) -> ProposalConfig:
        return ProposalConfig(self.consensus_threshold, self.max_rounds, self.use_gossipsub_rounds)


def resolve_config(base: ConsensusConfig, proposal: Proposal, explicit: bool = False) -> ConsensusConfig:
    """service.rs:444-484: timeout from the proposal's expiration unless explicitly overridden;
    liveness from the proposal."""
    timeout = base.consensus_timeout
    if not explicit and proposal.expiration_timestamp > proposal.timestamp:
        timeout = proposal.expiration_timestamp - proposal.timestamp
    return dataclasses.replace(base, consensus_timeout=timeout, liveness_criteria=proposal.liveness_criteria_yes)


@dataclass
class ProposalOutcome:
    """One proposal's result from the batch path: `error` is None on `Ok`, else the
    ConsensusError the reference returns; `transition` / `yes` / `total` are meaningful on Ok."""
    proposal_id: int
    error: Optional[errors.ConsensusError]
    transition: int = TRANSITION_STILL_ACTIVE
    consensus: Optional[bool] = None
    yes: int = 0
    total: int = 0
    bad_index: int = -1

    @property
    def ok(self) -> bool:
        return self.error is None


def _outcomes(proposals: Sequence[Proposal], res: np.ndarray) -> List[ProposalOutcome]:
    out = []
    for p, r in zip(proposals, res):
        st = int(r["status"])
        err = None if st == 0 else errors.from_status(st, int(r["scheme_reason"]))
        tr = int(r["transition"])
        cons = None
        if st == 0 and tr == 2:      # HLC_REACHED_YES
            cons = True
        elif st == 0 and tr == 1:    # HLC_REACHED_NO
            cons = False
        bad = int(r["bad_index"])
        out.append(ProposalOutcome(p.proposal_id, err, TRANSITION_CONSENSUS_REACHED if tr else TRANSITION_STILL_ACTIVE,
                                   cons, int(r["yes"]), int(r["total"]), bad if bad != 0xFFFFFFFF else -1))
    return out


def _device_scheme(scheme) -> bool:
    return scheme is None or getattr(scheme, "DEVICE_SCHEME", False)


def validate_batch(eng: Engine, batch, desc: np.ndarray, now: int, scheme=None) -> np.ndarray:
    """from_proposal over a packed batch under `scheme` (None: EthereumConsensusSigner) -> results."""
    if _device_scheme(scheme):
        res, _, _, _ = eng.validate_proposals(batch, desc, now, want_votes=False)
    else:
        verdicts = scheme_verdicts(scheme, batch, eng)
        res, _, _ = eng.validate_proposals_verdicts(batch, desc, now, verdicts, want_votes=False)
    return res


def validate_proposals(proposals: Sequence[Proposal], now: int, configs: Optional[Sequence[ConsensusConfig]] = None,
                       engine: Optional[Engine] = None, scheme=None) -> List[ProposalOutcome]:
    """Batched `ConsensusSession::from_proposal::<Signer>` validation (session.rs:198-300 incl.
    utils.rs:106-225): one GPU call for every proposal.  `scheme` is the `Signer` type (default
    EthereumConsensusSigner)."""
    eng = engine or Engine.default()
    cfgs = [(configs[i] if configs is not None else ConsensusConfig()).to_proposal_config() for i in range(len(proposals))]
    batch, desc = pack_proposals(proposals, cfgs)
    return _outcomes(proposals, validate_batch(eng, batch, desc, now, scheme))


def validate_proposal(proposal: Proposal, now: int, config: Optional[ConsensusConfig] = None,
                      engine: Optional[Engine] = None, scheme=None) -> ProposalOutcome:
    """utils.rs:106 + session.rs:198: raises the reference's ConsensusError on rejection."""
    o = validate_proposals([proposal], now, [config] if config else None, engine, scheme)[0]
    if o.error is not None:
        raise o.error
    return o


def compute_vote_hashes(votes: Sequence[Vote], engine: Optional[Engine] = None) -> List[bytes]:
    """utils.rs:37-52 over a batch (GPU SHA-256)."""
    eng = engine or Engine.default()
    if not votes:
        return []
    h = eng.compute_vote_hashes(pack_votes(votes))
    return [bytes(x) for x in h]


def compute_vote_hash(vote: Vote, engine: Optional[Engine] = None) -> bytes:
    return compute_vote_hashes([vote], engine)[0]


def build_vote(proposal: Proposal, vote: bool, signer, now: int, engine: Optional[Engine] = None) -> Vote:
    """utils.rs:55-104: chain onto the proposal's last vote, hash, sign (EIP-191) with `signer`."""
    from .protos import encode_vote
    owner = signer.identity()
    parent_hash = b""
    received_hash = b""
    if proposal.votes:
        received_hash = proposal.votes[-1].vote_hash
        for v in proposal.votes:
            if v.vote_owner == owner:
                parent_hash = v.vote_hash
    v = Vote(vote_id=_vote_id(owner, proposal.proposal_id, now), vote_owner=owner, proposal_id=proposal.proposal_id,
             timestamp=now, vote=vote, parent_hash=parent_hash, received_hash=received_hash)
    v.vote_hash = compute_vote_hash(v, engine)
    v.signature = signer.sign(encode_vote(v))
    return v


def _vote_id(owner: bytes, proposal_id: int, now: int) -> int:
    """The reference draws vote_id from `generate_id()` (utils.rs:79); any u32 is valid on the path."""
    import uuid
    return uuid.uuid4().int & 0xFFFFFFFF


@dataclass
class SessionRecord:
    """What the service keeps per accepted proposal (the subset of session.rs:160-190 the path
    produces): the proposal, the resolved config and the tally after initial validation."""
    proposal: Proposal
    config: ConsensusConfig
    transition: int
    consensus: Optional[bool]
    yes: int
    total: int
    created_at: int
    failed: bool = False       # ConsensusState::Failed (timeout without a result, round limit)
    round: int = 1             # Proposal.round of the session (session.rs:350-366)
    owners: set = field(default_factory=set)  # keys of the owner -> vote map

    @property
    def state(self) -> int:
        """HLC_SESSION_*: 0 Active, 1 ConsensusReached(false), 2 ConsensusReached(true), 3 Failed."""
        if self.consensus is not None:
            return 2 if self.consensus else 1
        return 3 if self.failed else 0


class ConsensusService:
    """service.rs:63-280 restricted to the incoming-proposal path (see module docstring)."""

    def __init__(self, engine: Optional[Engine] = None, default_config: Optional[ConsensusConfig] = None,
                 scheme=None):
        """`scheme`: the service's `Signer` type (service.rs:39-51), a ConsensusSignatureScheme subclass;
        None = EthereumConsensusSigner."""
        self.engine = engine or Engine.default()
        self.default_config = default_config or ConsensusConfig.gossipsub()
        self.scheme = scheme
        self.scope_configs: Dict[bytes, ConsensusConfig] = {}
        self.sessions: Dict[Tuple[bytes, int], SessionRecord] = {}

    def set_scope_config(self, scope: Union[str, bytes], config: ConsensusConfig) -> None:
        self.scope_configs[_scope_key(scope)] = config

    def get_session(self, scope: Union[str, bytes], proposal_id: int) -> SessionRecord:
        try:
            return self.sessions[(_scope_key(scope), proposal_id)]
        except KeyError:
            raise errors.SessionNotFound() from None

    def process_incoming_proposal(self, scope: Union[str, bytes], proposal: Proposal, now: int) -> None:
        """service.rs:263-279: raises the reference's error or stores the session."""
        o = self.process_incoming_proposals(scope, [proposal], now)[0]
        if o.error is not None:
            raise o.error

    def process_incoming_proposals(self, scope: Union[str, bytes], proposals: Sequence[Proposal],
                                   now: int) -> List[ProposalOutcome]:
        """The batched form the GPU path exists for: each proposal gets exactly the outcome the
        reference's per-proposal `process_incoming_proposal` returns when they are delivered in
        order.  A proposal id that is already stored (or repeats earlier in this batch) is
        rejected with ProposalAlreadyExist before validation, as service.rs:269-271 does."""
        key = _scope_key(scope)
        base = self.scope_configs.get(key, self.default_config)
        outcomes: List[Optional[ProposalOutcome]] = [None] * len(proposals)
        todo: List[int] = []
        seen = set()
        for i, p in enumerate(proposals):
            if (key, p.proposal_id) in self.sessions or p.proposal_id in seen:
                outcomes[i] = ProposalOutcome(p.proposal_id, errors.ProposalAlreadyExist())
            else:
                todo.append(i)
                seen.add(p.proposal_id)
        cfgs = [resolve_config(base, proposals[i]) for i in todo]
        sub = [proposals[i] for i in todo]
        if sub:
            res = validate_proposals(sub, now, cfgs, self.engine, self.scheme)
            # an id that fails validation is not stored, so a later copy in the batch would be
            # validated in the reference; re-run those (rare) in a second pass.
            retry: List[int] = []
            for i, cfg, o in zip(todo, cfgs, res):
                outcomes[i] = o
                if o.ok:
                    self._store(key, proposals[i], cfg, o, now)
            for i, p in enumerate(proposals):
                if outcomes[i] is not None and isinstance(outcomes[i].error, errors.ProposalAlreadyExist) \
                        and (key, p.proposal_id) not in self.sessions:
                    retry.append(i)
            if retry:
                for i in retry:
                    outcomes[i] = None
                rest = self.process_incoming_proposals(scope, [proposals[i] for i in retry], now)
                for i, o in zip(retry, rest):
                    outcomes[i] = o
        return outcomes  # type: ignore[return-value]

    def handle_consensus_timeout(self, scope: Union[str, bytes], proposal_id: int, now: int) -> bool:
        """service.rs:323-373: the consensus result, or raises InsufficientVotesAtTimeout (the
        session is then Failed) / SessionNotFound."""
        res = self.handle_consensus_timeouts(scope, [proposal_id], now)[0]
        if isinstance(res, errors.ConsensusError):
            raise res
        return res

    def handle_consensus_timeouts(self, scope: Union[str, bytes], proposal_ids: Sequence[int],
                                  now: int) -> List[Union[bool, errors.ConsensusError]]:
        """Batched timeout tally: one GPU call (hlc_consensus_timeout_batch) for every session;
        per id the result bool or the ConsensusError the reference returns."""
        from . import _ffi
        key = _scope_key(scope)
        recs = [self.sessions.get((key, pid)) for pid in proposal_ids]
        live = [r for r in recs if r is not None]
        arr = np.zeros(len(live), dtype=_ffi.SESSION_TALLY_DTYPE)
        for k, r in enumerate(live):
            arr[k]["total"], arr[k]["yes"] = r.total, r.yes
            arr[k]["expected_voters_count"] = r.proposal.expected_voters_count
            arr[k]["state"] = r.state
            arr[k]["liveness_criteria_yes"] = 1 if r.proposal.liveness_criteria_yes else 0
            arr[k]["consensus_threshold"] = r.config.consensus_threshold
        state, status = self.engine.consensus_timeout_batch(arr) if len(live) else (np.zeros(0), np.zeros(0))
        out: List[Union[bool, errors.ConsensusError]] = []
        k = 0
        for r in recs:
            if r is None:
                out.append(errors.SessionNotFound())
                continue
            st, code = int(state[k]), int(status[k])
            k += 1
            if code:
                r.failed = True
                out.append(errors.from_status(code))
            else:
                r.consensus = st == 2
                r.transition = TRANSITION_CONSENSUS_REACHED
                out.append(r.consensus)
        return out

    def process_incoming_vote(self, scope: Union[str, bytes], vote: Vote, now: int) -> None:
        """service.rs:286-305: raises the reference's error, else the vote is applied."""
        err = self.process_incoming_votes(scope, [vote], now)[0]
        if err is not None:
            raise err

    def process_incoming_votes(self, scope: Union[str, bytes], votes: Sequence[Vote],
                               now: int) -> List[Optional[errors.ConsensusError]]:
        """Micro-batched `process_incoming_vote`: one GPU call (hlc_process_votes) gives every vote
        exactly the outcome of the reference's calls in delivery order; None = Ok.  Accepted votes
        are appended to their session's proposal, states / rounds / tallies updated."""
        from . import _ffi
        key = _scope_key(scope)
        recs: List[SessionRecord] = []
        index: Dict[int, int] = {}
        vsess = np.full(len(votes), 0xFFFFFFFF, np.uint32)
        for i, v in enumerate(votes):
            r = self.sessions.get((key, v.proposal_id))
            if r is None:
                continue
            if v.proposal_id not in index:
                index[v.proposal_id] = len(recs)
                recs.append(r)
            vsess[i] = index[v.proposal_id]
        sarr = np.zeros(len(recs), _ffi.SESSION_DTYPE)
        orows, osess = [], []
        generic = not _device_scheme(self.scheme)
        for k, r in enumerate(recs):
            p, c = r.proposal, r.config
            sarr[k] = (p.timestamp, p.expiration_timestamp, p.proposal_id, p.expected_voters_count, r.round, r.total,
                       r.yes, c.max_rounds, c.consensus_threshold, r.state, int(c.use_gossipsub_rounds),
                       int(p.liveness_criteria_yes), (0,) * 5)
            for o in r.owners:
                if generic:
                    orows.append(bytes(o))
                    osess.append(k)
                elif len(o) == 20:  # (EthereumConsensusSigner admits only 20-byte identities)
                    orows.append(np.frombuffer(o, np.uint8))
                    osess.append(k)
        batch = pack_votes(votes)
        if generic:
            verdicts = scheme_verdicts(self.scheme, batch, self.engine)
            st, tr, ins, rs = self.engine.process_votes_verdicts(batch, vsess, sarr, orows, np.array(osess, np.uint32),
                                                                 now, verdicts)
        else:
            owners = np.stack(orows) if orows else np.zeros((0, 20), np.uint8)
            st, tr, ins, rs = self.engine.process_votes(batch, vsess, sarr, owners, np.array(osess, np.uint32), now)
        for k, r in enumerate(recs):
            s = sarr[k]
            r.round, r.total, r.yes = int(s["round"]), int(s["total"]), int(s["yes"])
            state = int(s["state"])
            r.failed = state == 3
            r.consensus = None if state in (0, 3) else state == 2
            if r.consensus is not None:
                r.transition = TRANSITION_CONSENSUS_REACHED
        out: List[Optional[errors.ConsensusError]] = []
        for i, v in enumerate(votes):
            if ins[i]:
                r = recs[int(vsess[i])]
                r.owners.add(v.vote_owner)
                r.proposal.votes.append(v)
            code = int(st[i])
            out.append(None if code == 0 else errors.from_status(code, int(rs[i])))
        return out

    def process_incoming_proposal_bytes(self, scope: Union[str, bytes], messages: Sequence[bytes],
                                        now: int) -> List[ProposalOutcome]:
        """Gossip bytes of Proposal messages -> outcomes, as if each were prost-decoded and passed
        to `process_incoming_proposal` in order.  Decoding runs on the device
        (hlc_decode_proposals); the decoded SoA batch goes straight to validate-many.  A message
        that does not decode gets ProposalDecodeError (the embedder's prost decode fails before
        service.rs:263); a stored id gets ProposalAlreadyExist (service.rs:269-271)."""
        from . import _ffi
        key = _scope_key(scope)
        base = self.scope_configs.get(key, self.default_config)
        lens = np.array([len(m) for m in messages], np.uint32)
        off = np.zeros(len(messages), np.uint64)
        if len(messages):
            off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
        wire = np.frombuffer(b"".join(messages), np.uint8)
        scope_cfg = np.zeros(1, _ffi.SCOPE_CONFIG_DTYPE)
        scope_cfg[0] = (base.consensus_threshold, base.max_rounds, int(base.use_gossipsub_rounds), (0, 0, 0))
        props, winfo, batch = self.engine.decode_proposals(wire, off, lens, scope_cfg)
        res = validate_batch(self.engine, batch, props, now, self.scheme)
        out: List[ProposalOutcome] = []
        for m, msg in enumerate(messages):
            if int(winfo[m]["decode_status"]) != 0:
                out.append(ProposalOutcome(0, errors.ProposalDecodeError()))
                continue
            p = _proposal_from_decoded(msg, props[m], winfo[m], batch, int(off[m]))
            if (key, p.proposal_id) in self.sessions:
                out.append(ProposalOutcome(p.proposal_id, errors.ProposalAlreadyExist()))
                continue
            o = _outcomes([p], res[m:m + 1])[0]
            out.append(o)
            if o.ok:
                self._store(key, p, resolve_config(base, p), o, now)
        return out

    def _store(self, key: bytes, p: Proposal, cfg: ConsensusConfig, o: ProposalOutcome, now: int) -> None:
        n = len(p.votes)
        rnd = (2 if n else 1) if cfg.use_gossipsub_rounds else min(1 + n, 0xFFFFFFFF)  # from_proposal: round 1 + update_round(n)
        self.sessions[(key, p.proposal_id)] = SessionRecord(p, cfg, o.transition, o.consensus, o.yes, o.total, now,
                                                            round=rnd, owners={v.vote_owner for v in p.votes})


def _proposal_from_decoded(msg: bytes, d, w, batch, base: int) -> Proposal:
    """Proposal object from the device decoder's outputs (hlc_proposal + hlc_wire_proposal +
    decoded vote SoA whose offsets index the wire buffer) -- marshalling only, no parsing."""
    def sl(o, n):
        return msg[int(o):int(o) + int(n)]
    votes = []
    for i in range(int(d["vote_begin"]), int(d["vote_begin"]) + int(d["vote_count"])):
        f = [batch.field(i, k) for k in range(5)]
        votes.append(Vote(vote_id=int(batch.vote_id[i]), vote_owner=f[0], proposal_id=int(batch.proposal_id[i]),
                          timestamp=int(batch.timestamp[i]), vote=bool(batch.vote[i]), parent_hash=f[1],
                          received_hash=f[2], vote_hash=f[3], signature=f[4]))
    return Proposal(name=sl(w["name_off"], w["name_len"]).decode("utf-8"), payload=sl(w["payload_off"], w["payload_len"]),
                    proposal_id=int(d["proposal_id"]), proposal_owner=sl(w["owner_off"], w["owner_len"]), votes=votes,
                    expected_voters_count=int(d["expected_voters_count"]), round=int(w["round"]),
                    timestamp=int(d["timestamp"]), expiration_timestamp=int(d["expiration_timestamp"]),
                    liveness_criteria_yes=bool(d["liveness_criteria_yes"]))


def _scope_key(scope: Union[str, bytes]) -> bytes:
    return scope.encode() if isinstance(scope, str) else bytes(scope)
