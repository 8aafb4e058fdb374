#!/usr/bin/env python3
"""Headline benchmark: verified votes/s of the batch vote-validation engine (BASELINE.json).

One "step" = one `hlc_validate_proposals_device` pass (the `ConsensusSession::from_proposal`
semantics of /root/reference/src/session.rs:198-221 for every proposal) over one batch of
synthetic signed votes already resident in HBM: SHA-256 vote-hash recompute, prost encoding,
EIP-191 keccak, secp256k1 ecrecover + address compare, timestamp checks, chain-link hash
table, duplicate-owner table, per-proposal tally/threshold/round limit.

Workload at N = 1 (the configuration BASELINE.json's metric is quoted
on): 10,000 proposals x 64 voters (Gossipsub, n = 64) = 640,000 votes per GPU, deterministic,
generated and signed on the GPU (hlc_synth_votes_device, bit-identical to synth.py).
At N > 1 (torch.distributed.run, one process per GPU, RCCL): config 4 -- rank r generates and
validates its own 1/8 shard of the 100M-vote workload (195,313 proposals x 64 = 12.5M votes), so
N = 8 is exactly config 4 (weak scaling, no data-path collective).  The one exchange per step is
the all_gather of the 16-byte per-proposal results plus an all_reduce(sum) of the verified /
rejected-by-code counters.

cpu_baseline: the C restatement of validate_vote (recover + k256's re-verify, as upstream) on
every host thread the process may use, one thread, and the two-pass (process_incoming_proposal)
rate, on rank 0, on a bounded sample of the same workload (at N > 1: of rank 0's shard, after the
timed region, the other ranks waiting at a barrier), and gpu_over_cpu for all N GPUs.
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
# Roofline constants frozen in roofline.json: the recovery is
# integer-VALU bound (no MFMA); W = 337,280 limb products per vote (canonical 8x32 CIOS
# ecrecover), peak = 39.3 T limb products/s (v_mad_u64_u32 at half rate: 4 cycles per wave64 against
# the 2-cycle VALU issue, 2.4 GHz); the VALU issue peak is 78.6 T lane-ops/s.
with open(os.path.join(ROOT, "roofline.json")) as _f:
    ROOFLINE = json.load(_f)
W_LIMB_PRODUCTS_PER_VOTE = ROOFLINE["W"]["limb_products_per_vote"]
MAD_PEAK_T_PER_S = ROOFLINE["peak"]["limb_products_T_per_s"]
W_IMPL_LIMB_PRODUCTS_PER_VOTE = ROOFLINE["implementation"]["limb_products_per_vote"]
# rocprofv3 passes of this bench (tools/profile.sh), committed under profiles/: kernel-trace
# summary, FETCH_SIZE / WRITE_SIZE and the VALU / wave counters of the recovery kernels.
PMC_PROFILE = os.path.join(ROOT, ROOFLINE["profile"])
# The recovery's kernels.  Round 6 on, the default schedule splits the u1 G comb off the finish
# (HLC_OPT_EARLY_COMB): k_rec_ucomb runs in k_rec_main's tail and k_rec_add adds u2 R after it; older
# profiles (and HLC_EARLY_COMB=0) hold the fused k_rec_comb instead.
REC_KERNELS_FUSED = ("k_rec_prep", "k_rec_main", "k_rec_comb", "k_rec_final", "k_rec_addr")
REC_KERNELS_EARLY = ("k_rec_prep", "k_rec_main", "k_rec_ucomb", "k_rec_add", "k_rec_final", "k_rec_addr")


def _profile_rec_kernels():
    path = os.path.join(PMC_PROFILE, "trace", "run_kernel_trace.csv")
    try:
        with open(path) as f:
            return REC_KERNELS_EARLY if "k_rec_ucomb(" in f.read() else REC_KERNELS_FUSED
    except OSError:
        return REC_KERNELS_EARLY


REC_KERNELS = _profile_rec_kernels()


def _pmc_rows(name: str):
    import csv
    path = os.path.join(PMC_PROFILE, name, "run_counter_collection.csv")
    if not os.path.exists(path):
        path = os.path.join(PMC_PROFILE, name + ".csv")
        if not os.path.exists(path):
            return []
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _is_kernel(name: str, kernel: str) -> bool:
    """Whether a trace row's Kernel_Name is `kernel` (a template instance such as k_rec_addr<true> too)."""
    return f"::{kernel}(" in name or f"::{kernel}<" in name


def pmc_per_launch(name: str, counter: str, kernel: str):
    """Average per launch of `counter` for `kernel` in the committed PMC pass `name`, or None."""
    vals = [float(r["Counter_Value"]) for r in _pmc_rows(name)
            if _is_kernel(r["Kernel_Name"], kernel) and r["Counter_Name"] == counter]
    return sum(vals) / len(vals) if vals else None


def pmc_duration_ms(name: str, kernel: str):
    """Average duration of `kernel` during the PMC pass `name` (its own dispatch timestamps)."""
    seen, durs = set(), []
    for r in _pmc_rows(name):
        if _is_kernel(r["Kernel_Name"], kernel) and r["Dispatch_Id"] not in seen:
            seen.add(r["Dispatch_Id"])
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return sum(durs) / len(durs) if durs else None


# Memory-side read bytes from the L2's request counters (round 4 doubled FETCH_SIZE for
# every kernel on the strength of the guide's note about 16-B-per-lane streams).  gfx950's FETCH_SIZE is
# (TCC_BUBBLE*128 + (TCC_EA0_RDREQ - TCC_BUBBLE - TCC_EA0_RDREQ_32B)*64 + TCC_EA0_RDREQ_32B*32) / 1024 KiB, and
# TCC_BUBBLE reads 0 on this box, so every request is tallied at 64 B.  Calibrated with tools/fetch_calib.hip
# (profiles/r05/fetch_calibration.json, fetch_calib_requests_by_size.csv: 2 GiB touched once per shape):
# every read request of every shape measured -- coalesced streams of 16-, 4- and 1-byte loads per lane, a
# lane's own 64-B entry at a scattered address (4 x 16-B loads), 32-B and 16-B pieces at scattered addresses --
# is a 128-B request (TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ; _64B and _32B ~0).  So the memory moves 128 B per
# request and FETCH_SIZE is exactly half of the memory-side read bytes for all of them; what differs by shape
# is the useful fraction: 1 for streams, 1/2 for 64-B gathers (the other half of the 128-B line comes along),
# 1/4 and 1/8 for 32- and 16-B pieces.  Read bytes per launch:
#   128 x TCC_EA0_RDREQ_128B + 64 x TCC_EA0_RDREQ_64B + 32 x TCC_EA0_RDREQ_32B   (pmc_req, when committed),
#   else 2 x FETCH_SIZE (the same for every shape calibrated), with FETCH_SIZE itself beside it.
REQ_COUNTERS = ("TCC_EA0_RDREQ", "TCC_EA0_RDREQ_128B", "TCC_EA0_RDREQ_32B")


def read_bytes(kernel: str, fetch_kib, req_pass: str = "pmc_req"):
    """(memory-side read bytes per launch, basis) for `kernel`: from the request-size pass when the
    committed profile has it, else 2 x FETCH_SIZE (see the calibration note above)."""
    req = {c: pmc_per_launch(req_pass, c, kernel) for c in REQ_COUNTERS}
    if all(v is not None for v in req.values()):
        rd, r128, r32 = (req[c] for c in REQ_COUNTERS)
        return 128.0 * r128 + 64.0 * (rd - r128 - r32) + 32.0 * r32, "request counters (pmc_req)"
    return 2.0 * fetch_kib * 1024.0, "2 x FETCH_SIZE (every calibrated read request is 128 B, tallied at 64 B)"


def pmc_traffic():
    """Per-launch memory-side bytes of the recovery kernels from the committed profile: reads by
    read_bytes() (the L2's read requests by size, or 2 x FETCH_SIZE), writes from WRITE_SIZE (exact for
    every shape calibrated, profiles/r05/fetch_calibration.json).  `fetch_raw_bytes` is FETCH_SIZE as
    counted; `fetch_x2_bytes` the round-4 blanket doubling, for comparison."""
    out = {}
    for k in REC_KERNELS:
        f = pmc_per_launch("pmc_fetch", "FETCH_SIZE", k)
        w = pmc_per_launch("pmc_write", "WRITE_SIZE", k)
        if f is None or w is None:
            return None
        rb, basis = read_bytes(k, f)
        out[k] = {"fetch_raw_bytes": f * 1024.0, "fetch_x2_bytes": 2.0 * f * 1024.0, "read_bytes": rb,
                  "read_basis": basis, "write_bytes": w * 1024.0}
    tot = {key: sum(v[key] for v in out.values()) for key in ("fetch_raw_bytes", "fetch_x2_bytes", "read_bytes",
                                                               "write_bytes")}
    tot["bytes"] = tot["read_bytes"] + tot["write_bytes"]
    tot["bytes_blanket_x2"] = tot["fetch_x2_bytes"] + tot["write_bytes"]
    tot["per_kernel"] = out
    tot["source"] = os.path.relpath(PMC_PROFILE, ROOT)
    tot["rule"] = ("reads: the L2's memory read requests by size (128 / 64 / 32 B; on gfx950 FETCH_SIZE tallies every "
                   "request at 64 B while every calibrated shape issues 128-B requests, tools/fetch_calib.hip); "
                   "writes: WRITE_SIZE")
    return tot


VALU_PEAK_LANE_OPS = ROOFLINE["peak"]["valu_lane_ops_T_per_s"]


def measure_live_clock(eng, step, torch):
    """The shader clock k_rec_main ran at on THIS box, right after the timed steps (the chip still in the
    state they left it in): three more steps with the library's per-wave clock stamps on
    (hlc_ctx_set_clock_probe; the timed steps ran without them), each call's median over its waves.
    Box-to-box differences in the headline follow this clock (MI355X_MICROARCH.md, DVFS give-back item 5);
    single calls can read well apart (2.26 then 1.94 GHz on one box), so all three are kept."""
    try:
        eng.set_clock_probe(True)
        calls = []
        for _ in range(3):
            step()
            torch.cuda.synchronize()
            calls.append(eng.clock_probe())
        meds = sorted(c["median_GHz"] for c in calls)
        return {"median_GHz": meds[1], "per_call_median_GHz": [c["median_GHz"] for c in calls],
                "min_GHz": min(c["min_GHz"] for c in calls), "max_GHz": max(c["max_GHz"] for c in calls),
                "waves_per_call": calls[-1]["waves"],
                "basis": "per-wave s_memtime / s_memrealtime over each k_rec_main wave's life; per call the "
                         "median over its waves; median_GHz = the middle of three calls right after the "
                         "timed steps"}
    except Exception as e:  # noqa: BLE001 -- a diagnostic, never the headline
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        try:
            eng.set_clock_probe(False)
        except Exception:  # noqa: BLE001
            pass


def valu_figures():
    """Hardware VALU figures of the recovery from the committed profile of this bench command
    (one build, one box): per kernel SQ_INSTS_VALU (PMC pass) x 64 lanes / its kernel-trace
    duration, against the guide's VALU issue peak (256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz =
    78.6 T lane-ops/s) -- `valu_lane_op_frac`, the figure the north star asks for; the issue
    fraction (SQ_INSTS_VALU per SIMD x the chain's measured 4.03 cycles per instruction over the
    kernel's GRBM cycles, both from the same PMC pass); and the clocks (PMC pass, in-kernel)."""
    insts = {k: pmc_per_launch("pmc_valu", "SQ_INSTS_VALU", k) for k in REC_KERNELS}
    grbm = pmc_per_launch("pmc_valu", "GRBM_GUI_ACTIVE", "k_rec_main")
    dur_pmc = pmc_duration_ms("pmc_valu", "k_rec_main")
    tr = rocprof_kernel_ms()
    if insts["k_rec_main"] is None or not grbm or not dur_pmc or not tr:
        return None
    hot = ROOFLINE["implementation"]["hot_op_issue"]
    simds, xcds = 256 * 4, 8
    cycles = grbm / xcds
    issue = insts["k_rec_main"] / simds * hot["cycles_per_wave_instruction"]
    pv = ROOFLINE["profile_votes_per_launch"]
    main_ms = tr["k_rec_main"]
    rate = insts["k_rec_main"] * 64.0 / (main_ms * 1e-3) / 1e12
    rec_insts = sum(v for v in insts.values() if v is not None)
    clk = ROOFLINE.get("measured_clock", {})
    return {
        "valu_instr_per_vote": {k: v * 64.0 / pv for k, v in insts.items() if v is not None},
        "valu_lane_op_rate_T": rate,
        "valu_lane_op_frac": rate / VALU_PEAK_LANE_OPS,
        "valu_lane_op_frac_basis": (f"k_rec_main: SQ_INSTS_VALU {insts['k_rec_main']:.4g} wave-instructions/launch "
                                    f"x 64 / {main_ms:.3f} ms (kernel-trace average of the timed steps) / "
                                    f"{VALU_PEAK_LANE_OPS} T lane-ops/s ({ROOFLINE['peak']['valu_basis']})"),
        "recovery_valu_instr_per_launch": rec_insts,
        "valu_issue_frac": issue / cycles,
        "pmc_pass_sclk_GHz": cycles / (dur_pmc * 1e6),
        "in_kernel_sclk_GHz": clk.get("k_rec_main_GHz"),
        "clock_ceiling_GHz": clk.get("point_op_loop_GHz"),
        "clock_source": clk.get("source"),
        "valu_issue_basis": (f"k_rec_main: SQ_INSTS_VALU / {simds} SIMDs x {hot['cycles_per_wave_instruction']} "
                             f"cycles/instruction ({hot['source']}) / {cycles:.4g} cycles (GRBM_GUI_ACTIVE per XCD, "
                             f"{dur_pmc:.3f} ms under PMC: profiled passes run at a lower clock, hence the separate "
                             f"in-kernel clock)"),
    }


def rocprof_kernel_ms():
    """Average durations (ms) of the recovery kernels over the timed steps of the committed
    kernel trace of this bench command (the last 20 validate-many calls), the recovery's critical
    path (`serial_chain_sum`: k_rec_prep's duration + k_rec_main's start to k_rec_addr's end -- the
    comb runs inside that span, after k_rec_main or in its tail) and the traced step period."""
    import csv
    import re
    import statistics
    path = os.path.join(PMC_PROFILE, "trace", "run_kernel_trace.csv")
    if not os.path.exists(path):
        return None
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            m = re.search(r"::(k_\w+)[(<]", r["Kernel_Name"])
            if m:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] == "k_rec_prep"]
    calls = []
    for ci, i0 in enumerate(starts):
        seg = rows[i0:starts[ci + 1] if ci + 1 < len(starts) else len(rows)]
        first = {}
        for t0, t1, k in seg:
            first.setdefault(k, (t0, t1))
        if all(k in first for k in REC_KERNELS):
            calls.append({k: (first[k][1] - first[k][0]) / 1e6 for k in REC_KERNELS}
                         | {"_t0": first["k_rec_prep"][0],
                            "_span": (first["k_rec_addr"][1] - first["k_rec_main"][0]) / 1e6})
    calls = calls[-20:]
    if not calls:
        return None
    out = {k: statistics.mean(c[k] for c in calls) for k in REC_KERNELS}
    out["serial_chain_sum"] = out["k_rec_prep"] + statistics.mean(c["_span"] for c in calls)
    out["traced_step_period"] = (statistics.mean((calls[i + 1]["_t0"] - calls[i]["_t0"]) / 1e6
                                                 for i in range(len(calls) - 1)) if len(calls) > 1 else None)
    out["calls"] = len(calls)
    out["source"] = os.path.relpath(path, ROOT)
    return out


CHAIN_KERNELS = ("k_chain_small", "k_clear_if", "k_tables", "k_chain_check", "k_vote_status", "k_finalize")
HBM_ACHIEVABLE_GBPS = 6290.0  # MI355X_MICROARCH.md: 8 TB/s spec, 6.29 TB/s measured (float4 copy)


def chain_counters(trace_dir: str, fetch_dir: str, write_dir: str):
    """Chain check + duplicate detection + tally kernels (validate_vote_chain utils.rs:175-215,
    initialize_with_votes session.rs:253-298, the tally utils.rs:227-286; k_vote_status's per-proposal
    first failing vote with them) per validate-many call, from the committed profile: each kernel's
    memory-side bytes (reads by read_bytes(): the L2's read requests by size, or 2 x FETCH_SIZE, the raw
    FETCH_SIZE beside it; WRITE_SIZE) over its own duration in a kernel trace where it runs alone (HLC_SERIAL_STAGES
    =1 for config 2, where k_chain_small otherwise shares the SIMDs with k_rec_main), and the achieved
    GB/s against the guide's measured 6.29 TB/s.  Per call = sum over the kernel's launches / the calls
    (k_finalize launches)."""
    import csv
    import re

    def rows(sub, fname):
        path = os.path.join(PMC_PROFILE, sub, fname)
        if not os.path.exists(path):
            return []
        with open(path, newline="") as f:
            return list(csv.DictReader(f))

    def kname(r):
        m = re.search(r"::(k_\w+)[(<]", r["Kernel_Name"])
        return m.group(1) if m else None

    tr = rows(trace_dir, "run_kernel_trace.csv")
    calls = sum(1 for r in tr if kname(r) == "k_finalize")
    if not calls:
        return None
    dur = {k: 0.0 for k in CHAIN_KERNELS}
    for r in tr:
        k = kname(r)
        if k in dur:
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    out = {}
    for sub, ctr in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        rr = rows(sub, "run_counter_collection.csv")
        pc = sum(1 for r in rr if kname(r) == "k_finalize" and r["Counter_Name"] == ctr)
        for k in CHAIN_KERNELS:
            v = sum(float(r["Counter_Value"]) for r in rr if kname(r) == k and r["Counter_Name"] == ctr) * 1024.0
            out.setdefault(k, {})[ctr] = v / max(pc, 1)
    per = {}
    tot_b = tot_raw = tot_ms = 0.0
    req_pass = fetch_dir.replace("fetch", "req")
    for k in CHAIN_KERNELS:
        f = out.get(k, {}).get("FETCH_SIZE", 0.0)
        w = out.get(k, {}).get("WRITE_SIZE", 0.0)
        ms = dur[k] / calls
        rb, basis = read_bytes(k, f / 1024.0, req_pass)
        b = rb + w
        per[k] = {"fetch_raw_bytes": f, "read_bytes": rb, "read_basis": basis, "write_bytes": w, "ms": ms,
                  "GBps": b / max(ms * 1e-3, 1e-12) / 1e9 if ms > 0 else None}
        tot_b += b
        tot_raw += f + w
        tot_ms += ms
    gbps = tot_b / max(tot_ms * 1e-3, 1e-12) / 1e9
    return {"bytes_per_call": tot_b, "bytes_per_call_raw_fetch": tot_raw, "isolated_ms_per_call": tot_ms,
            "GBps": gbps, "frac_of_hbm_achievable": gbps / HBM_ACHIEVABLE_GBPS, "per_kernel": per,
            "source": f"{os.path.relpath(PMC_PROFILE, ROOT)}/{{{trace_dir},{fetch_dir},{write_dir}}}"}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_quota():
    """Host CPUs this process may use: the affinity mask and, when set, the cgroup v2 quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return aff, quota


def physical_cores() -> int:
    """Physical cores of the host (distinct (physical id, core id) pairs of /proc/cpuinfo), not the
    CPUs this process may use."""
    try:
        pairs, phys = set(), None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":")[1].strip()
                elif line.startswith("core id"):
                    pairs.add((phys, line.split(":")[1].strip()))
        return len(pairs) or (os.cpu_count() or 1)
    except OSError:
        return os.cpu_count() or 1


def _cpulist(text: str) -> set:
    out = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def numa_facts(torch, dev, arrays) -> dict:
    """Where a host-buffer leg's memory and threads sit relative to the GPU: the
    GPU's NUMA node (sysfs, from its PCI address), the NUMA nodes of this process's CPUs, and the node
    of every page of the given numpy arrays (move_pages(2) with no target = query), as {node: pages}."""
    import ctypes
    out = {}
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            out["gpu_numa_node"] = int(f.read())
        out["gpu_pci"] = bdf
    except Exception as e:  # noqa: BLE001
        out["gpu_numa_node"] = f"unknown ({type(e).__name__})"
    try:
        aff = os.sched_getaffinity(0)
        nodes = {}
        base = "/sys/devices/system/node"
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                with open(f"{base}/{d}/cpulist") as f:
                    k = len(_cpulist(f.read()) & aff)
                if k:
                    nodes[int(d[4:])] = k
        out["process_cpus_by_node"] = nodes
    except OSError:
        pass
    try:
        import numpy as np
        libc = ctypes.CDLL(None, use_errno=True)
        pages = {}
        for a in arrays:
            lo = a.ctypes.data & ~4095
            n = (a.ctypes.data + a.nbytes - lo + 4095) // 4096
            step = max(1, n // 256)  # a sample of the array's pages
            addrs = np.arange(lo, lo + n * 4096, 4096 * step, dtype=np.uint64)
            st = np.zeros(addrs.size, np.int32)
            if libc.syscall(279, 0, ctypes.c_ulong(addrs.size), ctypes.c_void_p(addrs.ctypes.data), None,
                            ctypes.c_void_p(st.ctypes.data), 0) == 0:
                for v in st.tolist():
                    pages[v] = pages.get(v, 0) + 1
        out["input_pages_by_node"] = {str(k): v for k, v in sorted(pages.items())}
        out["pages_note"] = "sampled pages of the input arrays; negative = not resident (-errno)"
    except Exception as e:  # noqa: BLE001
        out["input_pages_by_node"] = f"unknown ({type(e).__name__})"
    return out


def traced_phases(eng, call, calls: int = 3) -> dict:
    """The host-buffer call's phase times (HLC_HOST_TRACE=2, hlc_ctx_last_host_trace) over `calls`
    extra untimed calls: per phase the median ms from the call's start, plus the trace's facts."""
    import statistics
    runs = []
    with eng.options(host_trace=2):  # HLC_OPT_HOST_TRACE: kept for hlc_ctx_last_host_trace only
        for _ in range(calls):
            call()
            runs.append(eng.last_host_trace())
    runs = [r for r in runs if r]
    if not runs:
        return {}
    med = lambda key: {k: statistics.median(r[key].get(k, float("nan")) for r in runs)  # noqa: E731
                       for k in runs[0][key]}
    return {"host_ms": med("host"), "device_ms": med("device"), "facts": runs[-1].get("facts", {}),
            "calls": len(runs), "what": "median over traced untimed calls; ms from the call's start (device: from "
                                        "an event recorded first on the upload stream)"}


def whole_host_estimate(single: float, per_thread: float) -> dict:
    """The CPU baseline scaled to every physical core of the host (keep the whole-host
    comparison visible beside the quota-bound one): the measured per-thread rate (the slower of the
    single-thread run and the quota run per thread) x physical cores, no SMT gain assumed."""
    cores = physical_cores()
    rate = min(single, per_thread)
    return {"value": rate * cores, "unit": "votes/s", "physical_cores": cores,
            "basis": "per-thread rate of this run x physical cores of the host (an estimate: linear scaling, "
                     "no SMT gain, no memory-bandwidth limit)"}


def cpu_baseline(batch, desc, now, sample_proposals: int, single_proposals: int) -> dict:
    """Times the oracle's C restatement (oracle/, the checker) on the host cores: the reference's
    per-vote validate_vote (utils.rs:127-171) with k256's recover + re-verify, on every host thread
    the process may use; the same on one thread; and the process_incoming_proposal-equivalent rate
    where from_proposal validates every vote twice (session.rs:203, 284-287).  The recovery timed is
    the k256-class path (hlc_oracle.c HLCO_GLV: GLV split, wNAF windows, binary-GCD inversions --
    k256 0.13.4 lincomb's algorithm class, /root/reference/Cargo.lock, called at
    src/signing/ethereum.rs:89); the independent non-GLV checker is timed beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402  (test infrastructure; cpu_baseline leg only)

    aff, quota = _cpu_quota()
    # every CPU the process may run on: the affinity mask, capped by the cgroup quota when one is set
    # (the GPU box grants 16 CPUs of a 256-thread host; 256 threads on 16 CPUs only time-slice --
    # measured 49.9k votes/s vs 79k with 16, profiles/r02_bench_cpu_threads.txt)
    threads = max(1, min(aff, int(quota + 0.999))) if quota else aff
    d_all = desc[:sample_proposals].copy()
    votes = int(d_all["vote_count"].sum())

    def timed(d, thr, passes=1, glv=True):
        t0 = time.perf_counter()
        for _ in range(passes):
            ok = coracle.validate_votes_only(batch, d, now, thr, reverify=True, glv=glv)
            assert ok == int(d["vote_count"].sum()), "CPU baseline rejected valid votes"
        return time.perf_counter() - t0

    dt = timed(d_all, threads)
    d1 = desc[:single_proposals].copy()
    v1 = int(d1["vote_count"].sum())
    dt1 = timed(d1, 1)
    dt2 = timed(d_all, threads, passes=2)
    d_chk = desc[:max(1, sample_proposals // 4)].copy()
    v_chk = int(d_chk["vote_count"].sum())
    dt_chk = timed(d_chk, threads, glv=False)
    return {
        "value": votes / dt,
        "unit": "votes/s",
        "cores": threads,
        "cores_note": ("threads = CPUs this process may use (affinity mask capped by the cgroup CPU quota); the "
                       "single-thread rate below scales the figure to any other core count"),
        "kind": "port",
        "algorithm": ("k256-class C restatement (oracle/hlc_oracle.c, HLCO_GLV): GLV split of both scalars (k256 "
                      "lincomb's decompose_scalar), wNAF windows of width 5 for R and 8 for G (odd-multiple tables "
                      "made affine by one inversion), binary extended-GCD inversions mod p and n, Jacobian "
                      "formulas, 4x64-bit limbs; k256's post-recovery verify_prehash kept (a second GLV "
                      "multiplication). Same outputs as the non-GLV checker on every item (tests/test_openssl_pin.py)"),
        "sample": f"{sample_proposals} proposals x {votes // max(sample_proposals, 1)} votes = {votes} votes of the "
                  f"same workload; validate_vote restated in C (SHA-256 + prost + EIP-191 keccak + ecrecover + "
                  f"k256 re-verify + timestamp checks), {threads} threads, {dt:.2f} s wall",
        "cpu_model": cpu_model(),
        "affinity_cpus": aff,
        "cgroup_cpu_quota": quota,
        "seconds": dt,
        "single_thread": {"value": v1 / dt1, "unit": "votes/s", "votes": v1, "seconds": dt1},
        "whole_host_estimate": whole_host_estimate(v1 / dt1, votes / dt / max(threads, 1)),
        "two_pass_rate": {"value": votes / dt2, "unit": "proposal votes/s", "votes": votes, "seconds": dt2,
                          "what": "process_incoming_proposal equivalent: every vote validated twice "
                                  "(validate_proposal + initialize_with_votes, session.rs:203, 284-287)"},
        "non_glv_checker": {"value": v_chk / dt_chk, "unit": "votes/s", "votes": v_chk, "threads": threads,
                            "seconds": dt_chk,
                            "algorithm": "4-bit Shamir windows without GLV, Fermat inversions (the independent "
                                         "checker; round 2's baseline)"},
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
    # the same bytes from host memory through hlc_validate_wire_proposals (upload, decode, validate,
    # per-proposal results back): what an embedder holding gossip bytes in host buffers sees
    host = None
    if dist is None:
        def host_call():
            return eng.validate_wire_proposals(wire, off, lens, scope, w.now)

        def timed_host():
            for _ in range(max(1, args.warmup)):
                host_call()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                hres, _, _ = host_call()
            assert np.array_equal(hres, res_s), "host wire-path outcomes differ from the SoA path"
            return (time.perf_counter() - t0) / args.steps

        hel = timed_host()
        # the unpipelined arm of the same entry (HLC_OPT_WIRE_PIPELINE 0: the whole buffer uploaded, then
        # decoded, then validated) beside it -- what the message-range pipeline gains
        with eng.options(wire_pipeline=0):
            pel = timed_host()
        host = {"value": db.n / hel, "unit": "votes/s", "ms_per_call": hel * 1e3,
                "what": "hlc_validate_wire_proposals from host buffers (PCIe-inclusive; pageable bytes, decoded and "
                        "recovered message range by message range as they land)",
                "unpipelined": {"value": db.n / pel, "unit": "votes/s", "ms_per_call": pel * 1e3,
                                "what": "the same entry with HLC_OPT_WIRE_PIPELINE 0 (upload all, decode, validate)"},
                "phases": traced_phases(eng, host_call)}
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
        **({"from_host_buffers": host} if host is not None else {}),
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


def e2e_leg(eng, w, args, np, torch, dev, pinned=False):
    """Secondary line: the same workload through the host-buffer entry hlc_validate_proposals
    (inputs copied host -> HBM over PCIe, results copied back, blocking): what a caller holding the
    votes in host memory sees.  Never the headline value (inputs are not HBM-resident).
    pinned=False: ordinary (pageable) numpy arrays, staged by the library's host pool into
    page-locked memory; pinned=True: the caller built its arrays in hlc_host_alloc memory, which
    the library DMAs with no staging copy (the batch is copied there once, before timing)."""
    b, d = w.batch, w.desc
    bytes_in = int(b.arena.nbytes + b.vote_id.nbytes + b.proposal_id.nbytes + b.timestamp.nbytes + b.vote.nbytes
                   + b.field_off.nbytes + b.field_len.nbytes + d.nbytes)
    if pinned:
        b = b.pinned()
    # the same warm-up for both legs (round 4 gave the page-locked leg one call only)
    for _ in range(max(1, args.warmup)):
        eng.validate_proposals(b, d, w.now, want_votes=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, vst, _, _ = eng.validate_proposals(b, d, w.now, want_votes=True)
    el = time.perf_counter() - t0
    assert (vst == 0).all() and (res["status"] == 0).all()
    return {
        "metric": ("verified votes/s, host buffers in and out (PCIe-inclusive hlc_validate_proposals)"
                   + (", inputs in page-locked memory (hlc_host_alloc)" if pinned else ", pageable inputs")),
        "value": b.n * args.steps / el,
        "unit": "votes/s",
        "ms_per_call": el / args.steps * 1e3,
        "bytes_in_per_call": bytes_in,
        "warmup_calls": max(1, args.warmup),
        "phases": traced_phases(eng, lambda: eng.validate_proposals(b, d, w.now, want_votes=True)),
        "numa": numa_facts(torch, dev, (b.arena, b.field_off, b.field_len, b.timestamp)),
    }


def e2e_leg_concurrent(eng, w, args, np, contexts: int = 3, threads: int = 4):
    """Secondary line: the host-buffer entry with `contexts` callers at once, one context and one
    thread each, every thread calling back to back on the same workload (include/hlc.h: one context
    per thread for concurrency) -- an embedder validating several proposal batches in parallel.  One
    call's lead-in (its first signatures' gather and upload) and its tail run beside the others'
    recovery, so the aggregate approaches the device-resident rate.  Aggregate votes/s over the
    slowest thread's time."""
    import threading

    from hashgraph_like_consensus.engine import Engine
    b, d = w.batch, w.desc
    old = eng.get_option("host_threads")
    engs = [eng] + [Engine(eng.device) for _ in range(contexts - 1)]
    for e in engs:
        e.set_option("host_threads", threads)  # HLC_OPT_HOST_THREADS per context
    try:
        for e in engs:
            e.validate_proposals(b, d, w.now, want_votes=True)
        go = threading.Barrier(contexts + 1)
        times = [0.0] * contexts
        bad = []

        def work(k):
            go.wait()
            try:
                t = time.perf_counter()
                for _ in range(args.steps):
                    res, vst, _, _ = engs[k].validate_proposals(b, d, w.now, want_votes=True)
                times[k] = time.perf_counter() - t
                if not ((vst == 0).all() and (res["status"] == 0).all()):
                    bad.append(k)
            except Exception as e:  # noqa: BLE001 -- re-raised on the calling thread below
                bad.append(f"{k}: {type(e).__name__}: {e}")

        th = [threading.Thread(target=work, args=(k,)) for k in range(contexts)]
        for x in th:
            x.start()
        go.wait()
        for x in th:
            x.join()
        assert not bad, f"contexts {bad}: failed or results differ from the expected outcomes"
        el = max(times)
    finally:
        for e in engs[1:]:
            e.close()
        eng.set_option("host_threads", old)
    return {
        "metric": "verified votes/s, host buffers in and out (PCIe-inclusive hlc_validate_proposals), "
                  f"{contexts} callers at once (one context + one thread each, {threads} staging threads per "
                  "context), aggregate",
        "value": contexts * args.steps * b.n / el,
        "unit": "votes/s",
        "contexts": contexts,
        "ms_per_call": el / args.steps * 1e3,
    }


def e2e_leg_sharded(eng, db, args, np, torch, dist, coll_dev, world):
    """Secondary line at N > 1 (end-to-end at 1/2/4/8 GPUs): every rank's shard
    through the host-buffer entry hlc_validate_proposals (its own votes copied to the host once,
    before timing: what a rank holding its shard in host memory sees), the same barrier + max-over-
    ranks timing as the headline, value = the votes all ranks processed / that time.  A failure on
    any rank (host memory, page-locked staging) is reported in the line instead of ending the run:
    every rank still takes part in the same collectives, so no rank is left waiting."""
    def agree(flag: bool) -> bool:  # True when every rank's flag is True
        t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    err = None
    try:
        b, d, _ = db.to_host()
        eng.validate_proposals(b, d, db.now, want_votes=True)
    except Exception as e:  # noqa: BLE001 -- reported in the line
        err = f"{type(e).__name__}: {e}"
    if not agree(err is None):
        return {"metric": "end-to-end (host-buffer) leg", "error": err or "failed on another rank"}
    dist.barrier()
    el, ok = 0.0, False
    try:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res, vst, _, _ = eng.validate_proposals(b, d, db.now, want_votes=True)
        el = time.perf_counter() - t0
        ok = bool((vst == 0).all() and (res["status"] == 0).all())
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    t = torch.tensor([el, 0.0 if ok else 1.0], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    nt = torch.tensor([b.n], dtype=torch.int64, device=coll_dev)
    dist.all_reduce(nt)
    if float(t[1].item()) != 0.0:
        return {"metric": "end-to-end (host-buffer) leg",
                "error": err or "a rank's host-buffer results differ from the expected outcomes"}
    el = float(t[0].item())
    return {
        "metric": "verified votes/s, host buffers in and out (PCIe-inclusive hlc_validate_proposals), every rank's "
                  "shard, pageable inputs",
        "value": int(nt.item()) * args.steps / el,
        "unit": "votes/s",
        "n_gpus": world,
        "ms_per_call": el / args.steps * 1e3,
        "votes_per_call_per_gpu": int(b.n),
    }


def config3_leg(eng, args, torch, synth, DeviceBatch, dev, ct):
    """Secondary line, SURVEY.md §8(d) config 3: one P2P proposal of 1,000,000 chained votes
    (n = 1.5M, so the ceil(2n/3) round cap is exactly 1M), generated on the device: the global
    chain / duplicate hash tables and the tally at scale.  Inputs resident in HBM, outcome asserted
    (every vote valid, the proposal OK with 1M votes) before the timed calls."""
    V = 1_000_000
    t = time.perf_counter()
    db = DeviceBatch.synthetic(eng, 1, V, 1_500_000, False, synth.config_seed(3), device=dev)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t
    eng.reserve(db.n, 1, db.bytes_len)
    s = torch.cuda.Stream(device=dev)
    eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    res = db.results_numpy()
    assert int(res["status"][0]) == 0 and int(res["total"][0]) == V and (db.status_numpy() == 0).all()
    eng.take_kernel_time()
    eng.take_chain_time()
    t = time.perf_counter()
    for _ in range(args.steps):
        eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / args.steps
    rec_ms, rec_n, _, _ = eng.take_kernel_time()
    ch_ms, ch_n = eng.take_chain_time()
    ch_s = ch_ms / max(ch_n, 1) / 1e3
    ch_bytes = ct["bytes_per_vote"] * V + ct["bytes_per_proposal"]
    return {
        "chain_tally_counters": chain_counters("c3_trace", "c3_fetch", "c3_write"),
        "metric": "verified votes/s, config 3 (1 P2P proposal, 1,000,000 chained votes, n = 1,500,000)",
        "value": V / el,
        "unit": "votes/s",
        "ms_per_call": el * 1e3,
        "recovery_ms": rec_ms / max(rec_n, 1),
        "chain_tally_ms": ch_s * 1e3,
        "chain_tally_GBps": ch_bytes / max(ch_s, 1e-12) / 1e9,
        "gen_seconds": gen_s,
    }


def config5_leg(eng, args, torch, synth, DeviceBatch, dev):
    """Secondary line, SURVEY.md §8(d) config 5: the config-2 shape with 1/3 Byzantine votes over
    17 mutation kinds, built on the device by product code (hlc_synth_byzantine_device: re-hashed
    and re-signed on the GPU).  Before timing, every per-vote status / scheme reason and every
    per-proposal first error is asserted equal to the outcome its mutation is built to have
    (hashgraph_like_consensus.byzantine, no oracle); the same batch is pinned to the C oracle bit for
    bit in tests/test_gpu_config5_device.py.  No short-circuit: every vote with a 65-byte signature
    is recovered, rejected or not."""
    import numpy as np
    from hashgraph_like_consensus import byzantine

    P, V = 10_000, 64
    seed = synth.config_seed(5)
    t = time.perf_counter()
    db = DeviceBatch.synthetic(eng, P, V, V, True, seed, device=dev)
    kinds = db.make_byzantine(eng, seed, 0)
    gen_s = time.perf_counter() - t
    assert np.array_equal(kinds, byzantine.plan(seed, 0, P, V)), "device mutation plan differs from the host plan"
    eng.reserve(db.n, P, db.bytes_len)
    s = torch.cuda.Stream(device=dev)
    eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    res, st = db.results_numpy(), db.status_numpy()
    rs = db.reason[: db.n].cpu().numpy()
    vst, vrs, pst, bad, yes, total = byzantine.expectations(kinds, V, db.choice_numpy())
    sch = st == byzantine.SCHEME
    assert np.array_equal(st, vst) and np.array_equal(rs[sch], vrs[sch]), "per-vote outcomes differ from construction"
    assert np.array_equal(res["status"], pst) and np.array_equal(res["bad_index"], bad), \
        "per-proposal first errors differ from construction"
    for _ in range(max(1, args.warmup)):
        eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        eng.validate_proposals_device(db, s.cuda_stream)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / args.steps
    assert np.array_equal(db.status_numpy(), vst)
    return {
        "metric": "verified votes/s, config 5 (config-2 shape, 1/3 Byzantine votes, bit-exact reject set)",
        "value": db.n / el,
        "unit": "votes/s",
        "ms_per_call": el * 1e3,
        "byzantine_votes": int((kinds != 0).sum()),
        "mutations_by_kind": {byzantine.NAMES[k]: int(c) for k, c in enumerate(np.bincount(kinds, minlength=18)) if k},
        "votes_by_status": byzantine.histogram(st),
        "proposals_by_status": byzantine.histogram(res["status"]),
        "outcomes_asserted": "per-vote status + scheme reason, per-proposal status + first bad index == construction",
        "gen_seconds": gen_s,
    }


CONFIG4_PROPOSALS = 1_562_500   # 100,000,000 votes = 1,562,500 x 64
CONFIG4_SHARDS = 8               # sharded by proposal over one 8-GPU node


def config4_shard(rank: int):
    """(first global proposal, count) of rank `rank`'s share of config 4 (8-way split)."""
    per = -(-CONFIG4_PROPOSALS // CONFIG4_SHARDS)
    start = min(rank * per, CONFIG4_PROPOSALS)
    return start, min(per, CONFIG4_PROPOSALS - start)


def config4_shard_leg(eng, args, torch, synth, DeviceBatch, dev):
    """Secondary line at N = 1: rank 0's shard of config 4 -- 195,313 proposals x 64 =
    12,500,032 votes, generated and signed on this GPU -- through exactly the per-rank step of the N > 1
    runs (hlc_validate_proposals_device + the outcome counters; the exchange has nothing to gather at one
    rank), so the driver's 1 -> 8 scaling curve has a same-workload N = 1 point (`scaling_basis`)."""
    from hashgraph_like_consensus.parallel import ShardExchange
    start, P = config4_shard(0)
    V = 64
    t = time.perf_counter()
    db = DeviceBatch.synthetic(eng, P, V, V, True, synth.config_seed(4), start_proposal=start, device=dev)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t
    eng.reserve(db.n, P, db.bytes_len)
    s = torch.cuda.Stream(device=dev)
    ex = ShardExchange(P, 1, dev, engine=eng)

    def step():
        eng.validate_proposals_device(db, s.cuda_stream)
        with torch.cuda.stream(s):
            ex.local_counters(db.results, db.status, P, db.n)

    step()
    torch.cuda.synchronize()
    res = db.results_numpy()
    assert (res["status"] == 0).all() and (res["total"] == V).all() and (db.status_numpy() == 0).all()
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / args.steps
    counters = ex.summary()
    assert counters["verified_votes"] == db.n
    n = db.n
    del db
    torch.cuda.empty_cache()
    return {
        "metric": "verified votes/s, config 4 rank-0 shard (195,313 proposals x 64 = 12.5M votes) on one GPU, "
                  "the per-rank step of the N > 1 runs",
        "value": n / el,
        "unit": "votes/s",
        "ms_per_step": el * 1e3,
        "votes_per_step": n,
        "proposals": P,
        "gen_seconds": gen_s,
    }


# the bench line printed on stdout carries the headline and one number per leg (a
# ~10 KB line was cut in the driver's tail); everything else -- phase traces, NUMA facts, per-kernel
# traffic, status histograms, rocprof kernel times -- goes to this side file, written by the same run
DETAIL_PATH = os.environ.get("HLC_BENCH_DETAIL") or os.path.join(ROOT, "profiles", "bench_detail.json")
LEG_NAMES = ("wire", "wire_from_host", "end_to_end", "end_to_end_pinned", "end_to_end_concurrent", "stream",
             "config3", "config5", "config4_shard")


def _value(d):
    return d.get("value") if isinstance(d, dict) else None


def compact_line(out: dict, detail_path: str) -> dict:
    """The stdout line from the full record: the driver's contract keys, a flat `legs` object of votes/s,
    the roofline and CPU-baseline essentials, and where the rest went (kept well under 4 KB)."""
    legs = {k: _value(out.get(k)) for k in LEG_NAMES}
    w = out.get("wire")
    if isinstance(w, dict):
        legs["wire_from_host"] = _value(w.get("from_host_buffers"))
    errors = {k: v["error"][:160] for k, v in out.items() if isinstance(v, dict) and "error" in v}
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config") if k in out}
    line["legs"] = {k: v for k, v in legs.items() if v is not None}
    if "scaling_basis" in out:
        line["scaling_basis"] = out["scaling_basis"]
    rf = out.get("roofline", {})
    live = rf.get("live_k_rec_main_clock") or {}
    line["roofline"] = {
        **{k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_per_vote",
                                  "frac_rocprof_chain", "valu_lane_op_frac", "valu_issue_frac", "kernel_ms_avg")},
        "kernel": "recovery: k_rec_prep + k_rec_main (+ k_rec_ucomb in its tail) + k_rec_add + k_rec_final + k_rec_addr (HIP events)",
        "valu_instr_per_vote_k_rec_main": (rf.get("valu_instr_per_vote") or {}).get("k_rec_main"),
        "live_k_rec_main_GHz": live.get("median_GHz"),
    }
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict) and "value" in cb:
        line["cpu_baseline"] = {**{k: cb.get(k) for k in ("value", "unit", "cores", "kind", "cpu_model")},
                                "sample": (cb.get("sample") or "")[:200],
                                "single_thread": _value(cb.get("single_thread")),
                                "whole_host_estimate": _value(cb.get("whole_host_estimate"))}
    for k in ("gpu_over_cpu", "gpu_over_cpu_whole_host_estimate", "counters_per_step", "gathered_results", "probe"):
        if k in out:
            line[k] = out[k]
    ct = out.get("chain_tally")
    if isinstance(ct, dict):
        line["chain_tally"] = {"ms_per_call": ct.get("ms_per_call"), "GBps": ct.get("GBps")}
    ex = out.get("exchange")
    if isinstance(ex, dict):
        line["exchange_ms_per_step"] = ex.get("ms_per_step_max_over_ranks")
    if errors:
        line["leg_errors"] = errors
    line["detail"] = os.path.relpath(detail_path, ROOT) if detail_path else None
    return line


def write_detail(out: dict, path: str):
    """The full record (every leg's phases, NUMA facts, traffic detail, histograms) as JSON; the path
    on success, None when it cannot be written (a read-only tree: the stdout line still prints)."""
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return path
    except OSError as e:
        print(f"bench: detail not written ({e})", file=sys.stderr, flush=True)
        return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, choices=[2, 4], default=None,
                    help="2: 10,000 x 64 votes per GPU (default at N=1); 4: this rank's 1/8 shard of the "
                         "100M-vote config 4, 195,313 x 64 votes (default at N>1)")
    ap.add_argument("--proposals", type=int, default=None, help="override the per-GPU proposal count")
    ap.add_argument("--votes-per-proposal", type=int, default=64)
    ap.add_argument("--cpu-sample-proposals", type=int, default=10_000)
    ap.add_argument("--cpu-single-proposals", type=int, default=250)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wire", action="store_true", help="skip the wire-bytes leg (device protobuf decode)")
    ap.add_argument("--no-stream", action="store_true", help="skip the streaming process_incoming_vote leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) leg")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 leg (1M-vote chain, ~10 s to generate)")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 leg (1/3 Byzantine votes)")
    ap.add_argument("--no-config4-shard", action="store_true",
                    help="skip the N = 1 config-4 shard leg (12.5M votes, the N > 1 per-rank workload)")
    args = ap.parse_args()

    import numpy as np
    import torch

    from hashgraph_like_consensus import synth
    from hashgraph_like_consensus.device import DeviceBatch, DeviceWire
    from hashgraph_like_consensus.engine import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # HLC_BENCH_BACKEND=gloo + HLC_BENCH_SAME_GPU=1: a dry run of the N > 1 path with every rank on
    # GPU 0 and the exchange over gloo on host copies (RCCL refuses two ranks on one GPU); the
    # driver's multi-GPU runs use the default, RCCL with one GPU per rank
    backend = os.environ.get("HLC_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("HLC_BENCH_SAME_GPU") == "1" else local_rank
    dist = None
    torch.cuda.set_device(gpu)
    # HLC_BENCH_DIST=1 at one rank: the N > 1 code path (process group, the RCCL exchange in the
    # timed step, the gathered-rows check) on one GPU -- the rehearsal of the driver's multi-GPU run
    if world > 1 or os.environ.get("HLC_BENCH_DIST") == "1":
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
        else:
            dist.init_process_group(backend)
    dev = f"cuda:{gpu}"
    coll_dev = dev if backend == "nccl" else "cpu"
    config = args.config or (2 if world == 1 else 4)

    eng = Engine(gpu)
    V = args.votes_per_proposal
    if config == 2:
        P = args.proposals or 10_000
        start, seed, max_p = rank * P, synth.config_seed(2), P
    else:
        start, P = config4_shard(rank)
        if args.proposals:
            P = args.proposals
            start = rank * P
        seed, max_p = synth.config_seed(4), max(config4_shard(r)[1] for r in range(max(world, 1)))
        max_p = max(max_p, P)
    # the workload is generated and signed on this rank's GPU (hlc_synth_votes_device, the synth.py
    # spec bit for bit): a rank builds only its own shard and nothing crosses PCIe
    t_gen = time.perf_counter()
    db = DeviceBatch.synthetic(eng, P, V, V, True, seed, start_proposal=start, device=dev)
    t_gen = time.perf_counter() - t_gen
    eng.reserve(db.n, P, db.bytes_len)
    stream = torch.cuda.Stream(device=dev)
    handle = stream.cuda_stream
    # the one exchange step (parallel.ShardExchange): every rank's 16-byte per-proposal
    # results all-gathered over RCCL plus an all_reduce(sum) of the verified / rejected-by-code
    # counters; at N = 1 only the local counters
    from hashgraph_like_consensus.parallel import ShardExchange
    ex = ShardExchange(max_p, world, coll_dev, engine=eng)

    ex_events = []  # (start, end) of the exchange on the launch stream, timed steps only

    def step(timed=False):
        eng.validate_proposals_device(db, handle)
        if dist is None:  # one GPU: the same outcome counters, on the device, with no exchange
            with torch.cuda.stream(stream):
                ex.local_counters(db.results, db.status, P, db.n)
        elif backend == "nccl":
            with torch.cuda.stream(stream):
                if timed:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                ex(db.results, db.status, P, db.n)
                if timed:
                    e1.record(stream)
                    ex_events.append((e0, e1))
        else:
            torch.cuda.synchronize()
            ex(db.results.cpu(), db.status.cpu(), P, db.n)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # guard: every synthetic vote is valid, every proposal validates (no silent breakage).  Timing
    # probe builds that compute wrong results on purpose (timing probes built with make variant) set
    # HLC_BENCH_PROBE=1, which skips the guard and marks the line as a probe.
    probe = os.environ.get("HLC_BENCH_PROBE") == "1"
    res = db.results_numpy()
    st = db.status_numpy()
    if not probe:
        assert (st == 0).all(), f"{int((st != 0).sum())} valid votes rejected"
        assert (res["status"] == 0).all() and (res["total"] == V).all()

    # the timed steps carry the recovery bracket only (two dispatch-bound events per call); the chain /
    # tally and whole-call brackets bind three more kernels on the critical path, so they are timed in
    # a pass of their own after the timed region (chain_pass below)
    eng.set_kernel_timing(True, recovery_only=True)
    eng.take_kernel_time()
    eng.take_chain_time()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rec_ms, rec_n, _, _ = eng.take_kernel_time()
    eng.set_kernel_timing(False)
    live_clock = measure_live_clock(eng, step, torch)
    # chain_pass: the same step, every bracket timed (chain check + duplicates + tally, the whole call)
    eng.set_kernel_timing(True)
    for _ in range(min(args.steps, 10)):
        step()
    torch.cuda.synchronize()
    _, _, call_ms, calls = eng.take_kernel_time()
    chain_ms, chain_n = eng.take_chain_time()
    eng.set_kernel_timing(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nt = torch.tensor([db.n], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(nt)
        votes_per_step = int(nt.item())
    else:
        votes_per_step = db.n
    counters = ex.summary()  # the last timed step's counters (all-reduced over the ranks at N > 1)
    if not probe:
        assert counters["verified_votes"] == votes_per_step, "all-reduced verified-vote counter != votes processed"
    gathered_check = None
    exchange = None
    if ex_events:
        # the exchange step's own time on the launch stream (counter kernel + all_gather + all_reduce),
        # max over ranks: what the collective adds to a step
        ms = sum(a.elapsed_time(b) for a, b in ex_events) / len(ex_events)
        t = torch.tensor([ms], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        exchange = {"ms_per_step_max_over_ranks": float(t.item()),
                    "bytes_gathered_per_step": int(ex.rows.numel()), "bytes_all_reduced_per_step": int(ex.counters.numel() * 8),
                    "what": "outcome-counter kernel + RCCL all_gather_into_tensor of the 16-B result rows + "
                            "all_reduce(sum) of the counters, HIP events on the launch stream"}
    if dist is not None:
        # the gathered per-proposal rows: every rank's slice of the all_gather equals that rank's own
        # results, byte for byte; the per-rank verdicts are all-reduced (MIN) so rank 0 reports all
        pc = torch.tensor([P], dtype=torch.int64, device=coll_dev)
        pcs = [torch.zeros_like(pc) for _ in range(world)]
        dist.all_gather(pcs, pc)
        counts = [int(x.item()) for x in pcs]
        rows = ex.results(counts)
        r0 = sum(counts[:rank])
        mine = np.array_equal(rows[r0:r0 + P].view(np.uint8), db.results_numpy().view(np.uint8))
        ok = torch.tensor([1 if mine else 0], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        gathered_check = {"rows": int(sum(counts)), "every_rank_slice_equals_local_results": bool(ok.item())}
        if not probe:
            assert gathered_check["every_rank_slice_equals_local_results"], "gathered result rows != local results"

    value = votes_per_step * args.steps / elapsed
    rec_avg_s = rec_ms / max(rec_n, 1) / 1e3
    achieved = W_LIMB_PRODUCTS_PER_VOTE * db.n / rec_avg_s / 1e12
    traffic = pmc_traffic()
    valu = valu_figures()
    rk = rocprof_kernel_ms()
    chain_avg_s = chain_ms / max(chain_n, 1) / 1e3
    ct = ROOFLINE["chain_tally"]
    chain_bytes = ct["bytes_per_vote"] * db.n + ct["bytes_per_proposal"] * P
    if config == 2:
        workload = (f"config2: {P} proposals x {V} voters (Gossipsub, n={V}) per GPU, full from_proposal validation"
                    if (P, V) == (10_000, 64) else
                    f"config2-shaped: {P} proposals x {V} voters (Gossipsub, n={V}) per GPU, full from_proposal "
                    f"validation")
    else:
        workload = (f"config4: rank shards of the 100M-vote workload (1,562,500 proposals x 64, 8-way split by "
                    f"proposal_id), {world} rank(s) = {votes_per_step:,} votes per step, full from_proposal validation")
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
            "workload": workload,
            "proposals_per_gpu": P,
            "votes_per_proposal": V,
            "votes_per_step_per_gpu": db.n,
            "votes_per_step": votes_per_step,
            "parallelism": f"proposal-sharded x{world}" + (
                f", {'RCCL' if backend == 'nccl' else backend} all_gather of results + all_reduce of counters"
                if world > 1 else ""),
        },
        "counters_per_step": counters,
        **({"gathered_results": gathered_check} if gathered_check is not None else {}),
        **({"exchange": exchange} if exchange is not None else {}),
        "roofline": {
            "bound": "valu",
            "kernel": ("recovery: k_rec_prep + k_rec_main (second stream, beside the prehash) + k_rec_ucomb (u1 G, in "
                       "k_rec_main's tail) + k_rec_add + k_rec_final + k_rec_addr (HIP-event brackets)"),
            "achieved": achieved,
            "peak": MAD_PEAK_T_PER_S,
            "unit": "T limb-products/s (32x32->64, v_mad_u64_u32)",
            "frac": achieved / MAD_PEAK_T_PER_S,
            "frac_basis": ("algorithmic: W limb products per vote x votes / the live recovery bracket / the "
                           "limb-product issue ceiling (roofline.json peak.basis); the hardware figure is "
                           "valu_lane_op_frac"),
            "frac_rocprof_chain": (W_LIMB_PRODUCTS_PER_VOTE * ROOFLINE["profile_votes_per_launch"]
                                   / (rk["serial_chain_sum"] * 1e-3) / 1e12 / MAD_PEAK_T_PER_S) if rk else None,
            "valu_lane_op_frac": valu["valu_lane_op_frac"] if valu else None,
            "valu_lane_op_rate_T": valu["valu_lane_op_rate_T"] if valu else None,
            "valu_lane_op_frac_basis": valu["valu_lane_op_frac_basis"] if valu else None,
            "valu_peak_lane_ops_T": VALU_PEAK_LANE_OPS,
            # per launch of THIS run: the profiled bytes per vote x this launch's votes
            "traffic": traffic["bytes"] / ROOFLINE["profile_votes_per_launch"] * db.n if traffic else None,
            "traffic_per_vote": traffic["bytes"] / ROOFLINE["profile_votes_per_launch"] if traffic else None,
            "traffic_detail": traffic,
            "work_per_vote": W_LIMB_PRODUCTS_PER_VOTE,
            "work_source": "roofline.json W (SURVEY.md 8(d): 2,480 modmul x 136 limb products, canonical algorithm)",
            "impl_work_per_vote": W_IMPL_LIMB_PRODUCTS_PER_VOTE,
            "impl_mad_pipe_frac": W_IMPL_LIMB_PRODUCTS_PER_VOTE * db.n / rec_avg_s / 1e12 / MAD_PEAK_T_PER_S,
            "valu_instr_per_vote": valu["valu_instr_per_vote"] if valu else None,
            "valu_issue_frac": valu["valu_issue_frac"] if valu else None,
            "valu_issue_basis": valu["valu_issue_basis"] if valu else None,
            "pmc_pass_sclk_GHz": valu["pmc_pass_sclk_GHz"] if valu else None,
            "in_kernel_sclk_GHz": valu["in_kernel_sclk_GHz"] if valu else None,
            "clock_ceiling_GHz": valu["clock_ceiling_GHz"] if valu else None,
            "live_k_rec_main_clock": live_clock,
            "clock_source": valu["clock_source"] if valu else None,
            "kernel_ms_avg": rec_avg_s * 1e3,
            "kernel_launches": rec_n,
            "rocprof_kernel_ms": rk,
            "call_ms_avg": call_ms / max(calls, 1),
            "kernel_share_of_step": (rec_ms / max(rec_n, 1)) / max(call_ms / max(calls, 1), 1e-9),
        },
        "chain_tally": {
            "what": "chain check + duplicate detection + tally kernels (utils.rs:175-286, session.rs:253-298), "
                    "HIP-event bracket per call (k_chain_small shares the SIMDs with k_rec_main here, so the "
                    "bracket is stretched; `counters` holds the isolated, counter-based figures)",
            "ms_per_call": chain_avg_s * 1e3,
            "bytes_per_call": chain_bytes,
            "GBps": chain_bytes / max(chain_avg_s, 1e-12) / 1e9,
            "bytes_model": ct["source"],
            "counters": chain_counters("trace_serial", "pmc_fetch", "pmc_write") if config == 2 else None,
        },
        "gen_seconds": t_gen,
    }
    need_host = world == 1 and ((not args.no_wire) or (not args.no_stream) or (not args.no_e2e) or
                                (rank == 0 and not args.no_cpu_baseline))
    w = None
    if need_host:
        hb, hd, _ = db.to_host()
        w = synth.Workload(hb, hd, db.now, None, "config%d" % config)
    def leg(name, fn):
        """A secondary leg: its failure is reported in the line (with the error) instead of losing
        the headline; only the headline's guard above ends the run."""
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001
            out[name] = {"error": f"{type(e).__name__}: {e}"}
            print(f"bench: leg {name} failed: {out[name]['error']}", file=sys.stderr, flush=True)

    if w is not None and not args.no_wire:
        leg("wire", lambda: wire_leg(eng, w, db, dev, stream, handle, args, world, dist, np, torch, synth, DeviceWire,
                                     elapsed / args.steps))
    if w is not None and not args.no_e2e:
        leg("end_to_end", lambda: e2e_leg(eng, w, args, np, torch, dev))
        leg("end_to_end_pinned", lambda: e2e_leg(eng, w, args, np, torch, dev, pinned=True))
        leg("end_to_end_concurrent", lambda: e2e_leg_concurrent(eng, w, args, np))
    if dist is not None and not args.no_e2e:
        out["end_to_end"] = e2e_leg_sharded(eng, db, args, np, torch, dist, coll_dev, world)
    if w is not None and not args.no_stream:
        leg("stream", lambda: stream_leg(eng, w, dev, stream, handle, args, world, dist, np, torch, DeviceBatch))
    if world == 1 and not args.no_config3:
        eng.set_kernel_timing(True)
        leg("config3", lambda: config3_leg(eng, args, torch, synth, DeviceBatch, dev, ct))
        eng.set_kernel_timing(False)
    if world == 1 and not args.no_config5:
        leg("config5", lambda: config5_leg(eng, args, torch, synth, DeviceBatch, dev))
    if world == 1 and not args.no_config4_shard:
        leg("config4_shard", lambda: config4_shard_leg(eng, args, torch, synth, DeviceBatch, dev))
    # what the per-GPU workload of each N is (the driver computes scaling from the per-N values)
    out["scaling_basis"] = {
        "n1_headline": "config 2: 640,000 votes per GPU per step (BASELINE.json configs[1])",
        "n_gt_1": "config 4 shards: 195,313 proposals x 64 = 12.5M votes per GPU per step",
        "n1_same_workload": "legs.config4_shard: rank 0's config-4 shard on one GPU, the per-rank step of N > 1",
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        leg("cpu_baseline", lambda: cpu_baseline(w.batch, w.desc, w.now, min(args.cpu_sample_proposals, P),
                                                 min(args.cpu_single_proposals, P)))
    elif dist is not None and not args.no_cpu_baseline:
        # N > 1: after the timed region and every collective of the legs above,
        # rank 0 times the same CPU baseline on a sample of its own shard (its first proposals, copied
        # back once) while the other ranks wait at a barrier; the line then states the north star's
        # ratio for all N GPUs
        if rank == 0:
            def cpu_leg():
                sample = min(args.cpu_sample_proposals, P)
                hb, hd = db.host_prefix(sample)
                cb = cpu_baseline(hb, hd, db.now, sample, min(args.cpu_single_proposals, sample))
                cb["timed_while"] = "the other ranks wait at a barrier (after the timed region)"
                return cb
            leg("cpu_baseline", cpu_leg)
        dist.barrier()
    if rank == 0 and "value" in out.get("cpu_baseline", {}):
        out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        out["gpu_over_cpu_whole_host_estimate"] = value / out["cpu_baseline"]["whole_host_estimate"]["value"]
        out["gpu_over_cpu_basis"] = (f"value ({world} GPU(s), all ranks' votes) / cpu_baseline.value "
                                     f"({out['cpu_baseline']['cores']} host threads)")
    if probe:
        out["probe"] = "HLC_BENCH_PROBE=1: a timing-probe build, results not checked (not a valid measurement)"
    if rank == 0:
        detail = write_detail(out, DETAIL_PATH)
        print(json.dumps(compact_line(out, detail)), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
