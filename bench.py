#!/usr/bin/env python3
"""Headline benchmark: verified votes/s of the batch vote-validation engine (BASELINE.json).

One "step" = one `hlc_validate_proposals_device` pass (the `ConsensusSession::from_proposal`
semantics of /root/reference/src/session.rs:198-221 for every proposal) over one batch of
synthetic signed votes already resident in HBM: SHA-256 vote-hash recompute, prost encoding,
EIP-191 keccak, secp256k1 ecrecover + address compare, timestamp checks, chain-link hash
table, duplicate-owner table, per-proposal tally/threshold/round limit.

Workload (the largest single-GPU config of BASELINE.json):
10,000 proposals x 64 voters (Gossipsub, n = 64) = 640,000 votes per GPU, deterministic,
generated and signed on the GPU by the engine's own signer (RFC 6979, EthereumConsensusSigner).
Multi-GPU (torch.distributed.run, one process per GPU, RCCL): every rank validates its own
proposal shard (weak scaling, no data-path collective); the per-proposal results (16 B each)
are all-gathered over RCCL once per step, the exchange the north star names.

cpu_baseline: the C restatement of validate_vote (recover + k256's re-verify, as upstream) on
the host cores, rank 0 at N = 1 only, on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))

METRIC = "verified votes/sec (ecrecover+chain check) at 1/2/4/8 MI355X vs host CPU"
# Roofline of the dominant kernel (k_recover, integer-VALU bound, no MFMA): its arithmetic is
# 32x32->64-bit limb products (v_mad_u64_u32).  Algorithmic work per vote, frozen in SURVEY.md
# §8(d) before tuning: 2,480 modmul x 136 limb products (canonical 8x32 Montgomery CIOS).
W_LIMB_PRODUCTS_PER_VOTE = 2480 * 136
# The implemented algorithm needs fewer (GLV + regular windows, 16-bit G comb, pseudo-Mersenne
# fold): DESIGN.md §5 counts its field operations -> reported beside, never as `achieved`.
W_IMPL_LIMB_PRODUCTS_PER_VOTE = 129_328
# Peak: v_mad_u64_u32 is quarter rate -- 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz
# (profiles/r01_ubench_int.txt measures 35.6 T/s).
MAD_PEAK_T_PER_S = 256 * 4 * 16 * 2.4e9 / 1e12
# rocprofv3 PMC passes of this same bench command (tools/profile.sh), committed under profiles/:
# `traffic` = memory-side bytes per k_recover launch from FETCH_SIZE / WRITE_SIZE (KiB), with the
# gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes).
PMC_PROFILE = os.path.join(ROOT, "profiles", "r01_rocprof_v13_s7")


def pmc_traffic(kernel: str = "k_recover"):
    """Per-launch (fetch, write, total) bytes of `kernel` from the committed PMC passes, or None."""
    import csv

    def per_launch(name: str, counter: str):
        path = os.path.join(PMC_PROFILE, name)
        if not os.path.exists(path):
            return None
        vals = []
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if f"::{kernel}(" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    vals.append(float(row["Counter_Value"]))
        return sum(vals) / len(vals) * 1024.0 if vals else None

    fetch = per_launch("pmc_fetch.csv", "FETCH_SIZE")
    write = per_launch("pmc_write.csv", "WRITE_SIZE")
    if fetch is None or write is None:
        return None
    fetch *= 2.0  # gfx950: FETCH_SIZE reports half the bytes of 128-B requests
    return {"fetch_bytes": fetch, "write_bytes": write, "bytes": fetch + write,
            "source": os.path.relpath(PMC_PROFILE, ROOT)}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(workload, sample_proposals: int) -> dict:
    """Times the oracle's C restatement (oracle/, the checker) on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402  (test infrastructure; cpu_baseline leg only)

    threads = max(1, min(16, os.cpu_count() or 1))
    desc = workload.desc[:sample_proposals].copy()
    votes = int(desc["vote_count"].sum())
    t0 = time.perf_counter()
    ok = coracle.validate_votes_only(workload.batch, desc, workload.now, threads, reverify=True)
    dt = time.perf_counter() - t0
    assert ok == votes, f"CPU baseline rejected {votes - ok} valid votes"
    return {
        "value": votes / dt,
        "unit": "votes/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample_proposals} proposals x {votes // max(sample_proposals, 1)} votes = {votes} votes of the "
                  f"same workload; validate_vote restated in C (SHA-256 + prost + EIP-191 keccak + ecrecover + "
                  f"k256 re-verify + timestamp checks), {threads} threads, {dt:.2f} s wall",
        "cpu_model": cpu_model(),
        "seconds": dt,
    }


def wire_leg(eng, w, db, dev, stream, handle, args, world, dist, np, torch, synth, DeviceWire, soa_step_s):
    """Secondary line: the same proposals as gossip bytes -- one prost
    `Proposal` message each, votes embedded -- resident in HBM, decoded on the device and fed to
    the same validation pipeline (hlc_validate_wire_proposals_device).  Also the full-size
    property check: wire-path outcomes == SoA-path outcomes for every proposal."""
    t0 = time.perf_counter()
    wire, off, lens, scope = synth.to_wire(w.batch, w.desc)
    t_enc = time.perf_counter() - t0
    dw = DeviceWire(wire, off, lens, scope, w.now, device=dev)

    def step():
        eng.validate_wire_proposals_device(dw, handle)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    res_w, res_s = dw.results_numpy(), db.results_numpy()
    assert np.array_equal(res_w, res_s), "wire-path outcomes differ from the SoA path"
    assert (dw.winfo_numpy()["decode_status"] == 0).all()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    step_s = el / args.steps
    return {
        "metric": "verified votes/s from wire bytes (device protobuf decode + validation)",
        "value": db.n * world * args.steps / el,
        "unit": "votes/s",
        "ms_per_step": step_s * 1e3,
        "wire_bytes_per_step_per_gpu": int(wire.size),
        "decode_overhead_ms": (step_s - soa_step_s) * 1e3,
        "decode_overhead_GBps": wire.size / max(step_s - soa_step_s, 1e-9) / 1e9,
        "outcomes_equal_soa_path": True,
        "host_encode_seconds": t_enc,
    }


def stream_leg(eng, w, dev, stream, handle, args, world, dist, np, torch, DeviceBatch):
    """Secondary line: the same 640k signed votes delivered one by one to 10k
    live sessions (fresh: no votes yet), in a shuffled gossip order, as micro-batched
    `process_incoming_vote` calls (hlc_process_votes_device, inputs in HBM).  Each step restores
    the initial sessions (a 560 KB device copy, inside the timed region) and processes every vote:
    validate_vote on the GPU, then add_vote per session in delivery order.  Consistency guard:
    every vote validates, and the votes marked inserted add up to the sessions' final totals."""
    from hashgraph_like_consensus import _ffi
    from hashgraph_like_consensus.batch import VoteBatch

    b, d = w.batch, w.desc
    P = d.shape[0]
    perm = np.random.default_rng(0x484C4302).permutation(b.n)
    pb = VoteBatch(vote_id=b.vote_id[perm], proposal_id=b.proposal_id[perm], timestamp=b.timestamp[perm],
                   vote=b.vote[perm], arena=b.arena, field_off=b.field_off[perm], field_len=b.field_len[perm])
    vsess = np.repeat(np.arange(P, dtype=np.uint32), d["vote_count"].astype(np.int64))[perm]
    sess = np.zeros(P, _ffi.SESSION_DTYPE)
    for f in ("timestamp", "expiration_timestamp", "proposal_id", "expected_voters_count", "max_rounds",
              "consensus_threshold", "use_gossipsub_rounds", "liveness_criteria_yes"):
        sess[f] = d[f]
    sess["round"] = 1
    dpb = DeviceBatch(pb, d, w.now, device=dev)
    t_vs = torch.from_numpy(vsess.view(np.uint8).copy()).to(dev)
    t_init = torch.from_numpy(sess.view(np.uint8).reshape(-1).copy()).to(dev)
    t_sess = t_init.clone()
    n = pb.n
    outs = [torch.zeros(n + 1, dtype=torch.uint8, device=dev) for _ in range(3)]

    def step():
        with torch.cuda.stream(stream):
            t_sess.copy_(t_init)
        eng.process_votes_device(dpb, t_vs.data_ptr(), t_sess.data_ptr(), P, w.now, outs[0].data_ptr(),
                                 outs[1].data_ptr(), outs[2].data_ptr(), handle)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    st = outs[0][:n].cpu().numpy()
    ins = outs[2][:n].cpu().numpy()
    fin = t_sess.cpu().numpy().view(_ffi.SESSION_DTYPE)
    assert (st == 0).all(), f"{int((st != 0).sum())} streamed votes rejected"
    assert int(ins.sum()) == int(fin["total"].sum()) and (fin["state"] != 3).all()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return {
        "metric": "incoming votes/s, micro-batched process_incoming_vote (validate_vote + add_vote per session)",
        "value": n * world * args.steps / el,
        "unit": "votes/s",
        "ms_per_step": el / args.steps * 1e3,
        "votes_per_step_per_gpu": n,
        "sessions": P,
        "inserted_per_step": int(ins.sum()),
        "decided_sessions": int((fin["state"] != 0).sum()),
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--proposals", type=int, default=10_000)
    ap.add_argument("--votes-per-proposal", type=int, default=64)
    ap.add_argument("--cpu-sample-proposals", type=int, default=10_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wire", action="store_true", help="skip the wire-bytes leg (device protobuf decode)")
    ap.add_argument("--no-stream", action="store_true", help="skip the streaming process_incoming_vote leg")
    args = ap.parse_args()

    import numpy as np
    import torch

    from hashgraph_like_consensus import synth
    from hashgraph_like_consensus.device import DeviceBatch, DeviceWire
    from hashgraph_like_consensus.engine import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    else:
        torch.cuda.set_device(local_rank)
    dev = f"cuda:{local_rank}"

    eng = Engine(local_rank)
    P, V = args.proposals, args.votes_per_proposal
    t_gen = time.perf_counter()
    addr_fn, sign_fn = synth.engine_signers(eng)
    w = synth.generate(P, V, V, True, synth.config_seed(2), addr_fn, sign_fn, start_proposal=rank * P,
                       name="config2")
    t_gen = time.perf_counter() - t_gen
    db = DeviceBatch(w.batch, w.desc, w.now, device=dev)
    eng.reserve(db.n, P, int(w.batch.arena.size))
    stream = torch.cuda.Stream(device=dev)
    handle = stream.cuda_stream
    gathered = None
    if dist is not None:
        gathered = [torch.empty_like(db.results) for _ in range(world)]

    def step():
        eng.validate_proposals_device(db, handle)
        if dist is not None:
            with torch.cuda.stream(stream):
                dist.all_gather(gathered, db.results)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # guard: every synthetic vote is valid, every proposal validates (no silent breakage)
    res = db.results_numpy()
    st = db.status_numpy()
    assert (st == 0).all(), f"{int((st != 0).sum())} valid votes rejected"
    assert (res["status"] == 0).all() and (res["total"] == V).all()

    eng.set_kernel_timing(True)
    eng.take_kernel_time()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rec_ms, rec_n, call_ms, calls = eng.take_kernel_time()
    eng.set_kernel_timing(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    votes_total = db.n * world * args.steps
    value = votes_total / elapsed
    rec_avg_s = rec_ms / max(rec_n, 1) / 1e3
    achieved = W_LIMB_PRODUCTS_PER_VOTE * db.n / rec_avg_s / 1e12
    traffic = pmc_traffic("k_recover")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "votes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: deterministic signed votes (SURVEY §8d spec), generated + RFC6979-signed on the GPU",
        "config": {
            "workload": (f"config2: {P} proposals x {V} voters (Gossipsub, n={V}) per GPU, full from_proposal validation"
                         if (P, V) == (10_000, 64) else
                         f"config2-shaped: {P} proposals x {V} voters (Gossipsub, n={V}) per GPU, full from_proposal "
                         f"validation" + (" (one rank's shard of config 4, 100M votes / 8 GPUs)" if P == 195_313 else "")),
            "proposals_per_gpu": P,
            "votes_per_proposal": V,
            "votes_per_step_per_gpu": db.n,
            "parallelism": f"proposal-sharded x{world}" + (", RCCL all_gather of results" if world > 1 else ""),
        },
        "roofline": {
            "bound": "valu",
            "kernel": "k_recover",
            "achieved": achieved,
            "peak": MAD_PEAK_T_PER_S,
            "unit": "T limb-products/s (32x32->64, v_mad_u64_u32)",
            "frac": achieved / MAD_PEAK_T_PER_S,
            "traffic": traffic["bytes"] if traffic else None,
            "traffic_detail": traffic,
            "work_per_vote": W_LIMB_PRODUCTS_PER_VOTE,
            "work_source": "SURVEY.md 8(d): 2,480 modmul x 136 limb products (canonical algorithm)",
            "impl_work_per_vote": W_IMPL_LIMB_PRODUCTS_PER_VOTE,
            "impl_mad_pipe_frac": W_IMPL_LIMB_PRODUCTS_PER_VOTE * db.n / rec_avg_s / 1e12 / MAD_PEAK_T_PER_S,
            "kernel_ms_avg": rec_avg_s * 1e3,
            "kernel_launches": rec_n,
            "call_ms_avg": call_ms / max(calls, 1),
            "kernel_share_of_step": rec_ms / max(call_ms, 1e-9),
        },
        "gen_seconds": t_gen,
    }
    if not args.no_wire:
        out["wire"] = wire_leg(eng, w, db, dev, stream, handle, args, world, dist, np, torch, synth, DeviceWire,
                               elapsed / args.steps)
    if not args.no_stream:
        out["stream"] = stream_leg(eng, w, dev, stream, handle, args, world, dist, np, torch, DeviceBatch)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(w, min(args.cpu_sample_proposals, P))
        out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
