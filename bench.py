#!/usr/bin/env python3
"""Headline benchmark: Groth16 proofs/s for the Venmo-shaped circuit on MI355X.

BASELINE.json metric: "Groth16 proofs/sec (node) + 1-proof latency, Venmo circuit;
G1 MSM Mpts/s".  Workload at N=1 = configs[2] (full Venmo-circuit proof on one
MI355X); the circuit is SYNTHETIC with the Venmo shape (nVars 6,400,562,
nConstraints 6,618,823, nPublic 26, domain 2^23) because the
real 3.5 GB zkey / witness are absent.  Insecure known-tau setup.

A "step" = one complete proof (buildABC, 3 coset NTTs, joinABC, 4 G1 + 1 G2 MSMs,
blinding) of one distinct synthetic witness already resident in HBM (staged).

Multi-GPU = replicas, no collectives (SURVEY.md §8e E1(1), configs[3]); value = all
proofs / wall time (max over ranks), n_gpus = devices actually used:
  * `torchrun --nproc-per-node N bench.py --gpus N`: one process per GPU (LOCAL_RANK),
    each with its own resident key; gloo carries only the barrier and the max.
  * `python bench.py --gpus N` (no torchrun): ONE process, one resident prover over
    devices [0..N-1] (zkp_prover_load with N devices), one host thread per device running
    staged proofs concurrently.  Fewer than N visible devices -> exit status 2 with a
    message, never a silent 1-GPU line.  `--rehearsal` maps the N logical devices onto
    device 0 (pipelines sharing one copy of the base tables) and marks the line
    "rehearsal": true -- a check of the multi-device code path, not a scaling number.
Every timed proof and every batch proof is compared with a separately computed proof of
the same witness at the same r, s.  Extra fields: latency, per-stage ms, config-1 kernels
(G1 MSM 2^20 Mpts/s, Fr NTT 2^20 / 2^23), roofline of the bucket-accumulate kernel (HIP
events), and the C++ CPU restatement (oracle/cpu) timed on this host as cpu_baseline.
"""
import argparse
import ctypes
import gc
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))

import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402

CIRCUIT_SEED = 0x5A4B5032
SETUP_SEED = 0x5A4B5033
# Measured on MI355X by tools/ubench/int_mul_rate (profiles/ubench_r01.txt): v_mad_u64_u32
# throughput, the instruction every 32x32->64 partial product of the field multiply maps to.
MAD_PEAK_TOPS = None  # filled from profiles/ubench_r01.json when present
MAC_PER_FPMUL = 136     # SURVEY.md §8d D4 (8x32-bit CIOS: 64 + 64 + 8)
FPMUL_PER_MADD = 11     # SURVEY.md §8d D4 (mixed Jacobian add 7M + 4S)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# one wave64 v_mad_u64_u32 per SIMD per quad-cycle (4 clocks) at 2.4 GHz: the 4-clock class, which is every
# instruction of the field products; the 2-clock class (v_and/add/sub/mov/lshrrev_b32 e32) shares a quad-cycle
# only with another wave's 2-clock instruction (profiles/valu_rates_r06.txt, profiles/pmc_valu_r06.json)
ISSUE_CEILING_TOPS = 256 * 64 * 2.4e9 / 1e12


def load_peak():
    """The measured v_mad_u64_u32 peak: profiles/ubench_r05.json (the best row of the occupancy sweep it
    lists, tools/ubench/int_mul_rate.hip), else round 1's summary."""
    for name in ("ubench_r05.json", "ubench_r01.json"):
        p = os.path.join(ROOT, "profiles", name)
        try:
            with open(p) as f:
                return json.load(f)["v_mad_u64_u32_tops"], os.path.relpath(p, ROOT)
        except Exception:
            continue
    return None, None


def load_ntt_issue():
    """Counted NTT issue figures of the current library (profiles/ntt_issue_r05.json, its "current" entry per size:
    273c6e8:tools/gpu/r5/pmc.sh, ntt_root1.sh)."""
    try:
        with open(os.path.join(ROOT, "profiles", "ntt_issue_r05.json")) as f:
            d = json.load(f)
        return {k: v.get(d.get("current", "cur")) for k, v in d["sizes"].items()}
    except Exception:
        return {}


def load_valu_counted():
    """Counted VALU busy per launch kind (profiles/pmc_valu_r06.json, tools/prof/valu_counted.py): the VALU's busy
    quad-cycles are SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2 (two full-rate instructions of two waves share one
    quad-cycle; every other VALU instruction takes one), over 1024 SIMDs x the launch's own clock."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_valu_r06.json")) as f:
            d = json.load(f)
        return {k: v["valu_busy_counted"] for k, v in d["accumulate"].items()}
    except Exception:
        return {}


def load_traffic():
    """Newest committed PMC summary of the accumulate kernel.  HBM bytes per launch = FETCH_SIZE +
    WRITE_SIZE: the kernel's bytes are random 64-B base gathers, for which FETCH_SIZE counts the
    bytes exactly (profiles/fetch_calibration_r02.json; the x2 of coalesced 16-B streams does not
    apply).  Round 4's summary is per launch kind (the H launch, the roofline's); older summaries
    averaged every G1 launch and are recomputed from their raw counters."""
    for name in ("pmc_launch_r06.json", "pmc_launch_r05.json"):
        p = os.path.join(ROOT, "profiles", name)
        if os.path.exists(p):
            break
    try:
        with open(p) as f:
            d = json.load(f)
        h = d["kinds"]["H"]
        return {"hbm_bytes_per_launch": h["hbm_bytes_per_dispatch"],
                "valu_lane_instructions_per_addition": h["valu_lane_instructions_per_addition"],
                "valu_issue_frac": h["valu_issue_frac"], "clock_GHz": h["clock_GHz"],
                "per_kind": {k: {"valu_issue_frac_pmc": v["valu_issue_frac"], "clock_GHz_pmc": v["clock_GHz"],
                                 "valu_lane_instructions_per_addition_pmc": v["valu_lane_instructions_per_addition"],
                                 "hbm_bytes_per_addition_pmc": v.get("hbm_bytes_per_addition")}
                             for k, v in d["kinds"].items()},
                "source": "profiles/%s (the H launch: rocprofv3 --pmc FETCH_SIZE x1 + WRITE_SIZE, "
                          "gather-calibrated; SQ_INSTS_VALU and GRBM_GUI_ACTIVE: issue share at the launch's own clock; "
                          "tools/prof/pmc_launch5.py)" % name}
    except Exception:
        pass
    p = os.path.join(ROOT, "profiles", "pmc_launch_r04.json")
    try:
        with open(p) as f:
            h = json.load(f)["kinds"]["H"]
        return {"hbm_bytes_per_launch": h["hbm_bytes_per_dispatch"],
                "valu_lane_instructions_per_addition": h.get("valu_lane_instructions_per_addition"),
                "source": "profiles/pmc_launch_r04.json (the H launch: rocprofv3 --pmc FETCH_SIZE x1 + WRITE_SIZE, "
                          "gather-calibrated; tools/prof/pmc_launch.py)"}
    except Exception:
        pass
    for name in ("pmc_accumulate_r03.json", "pmc_accumulate_r02.json", "pmc_accumulate_r01.json"):
        p = os.path.join(ROOT, "profiles", name)
        try:
            with open(p) as f:
                d = json.load(f)
        except Exception:
            continue
        g1 = d.get("kernels", {}).get("k_accumulate<Fq >") or d.get("kernels", {}).get("k_accumulate<Fq>")
        if g1:
            d["hbm_bytes_per_launch"] = (g1["FETCH_SIZE_kb_avg"] + g1["WRITE_SIZE_kb_avg"]) * 1024
        d["source"] = "profiles/%s (rocprofv3 --pmc FETCH_SIZE x1 + WRITE_SIZE per launch, gather-calibrated)" % name
        return d
    return None


def gen_witnesses(circ, seeds):
    out = [None] * len(seeds)

    def work(i):
        out[i] = circ.witness(seeds[i])

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(seeds))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return out


def visible_devices():
    """GPUs this process can use (counting does not initialise the GPU on this image)."""
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def host_cpu_info():
    """What the CPU baseline runs on: `nproc` (CPUs this process may run on), the machine's
    logical CPU count, the cgroup CPU quota (cores) if one is set, and the CPU model."""
    try:
        nproc = len(os.sched_getaffinity(0))
    except Exception:
        nproc = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    usable = nproc if quota is None else max(1, min(nproc, int(quota + 0.5)))
    return {"nproc": nproc, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota_cores": quota,
            "cpu_model": model, "usable_cores": usable}


PUBLISHED_CPU = {  # BASELINE.md (reference zkp-mooc-hackathon-submission.md:89,92,101): whole Venmo proof
    "rapidsnark_s_per_proof": 9.2, "rapidsnark_hardware": "AWS z1d.12xlarge, 48 vCPU",
    "snarkjs_browser_s_per_proof": 623.0, "source": "zkp-mooc-hackathon-submission.md:89,101 (published, other hardware)"}


def kernel_benches(device, log_n=20, iters=10):
    """configs[1]: G1 MSM 2^20 (uniform scalars) + Fr NTT 2^20, device-resident.  The MSM
    result is cross-checked against the same MSM with different Pippenger parameters (window
    13 bits, no precomputed rows: other plan, other buckets, host Horner over the windows)."""
    n = 1 << log_n
    sc_pts = synth.scalars(CIRCUIT_SEED, 0, n)
    pts = synth.points(sc_pts, g2=False, device=device)
    scal = synth.scalars(CIRCUIT_SEED, 1, n)
    st, res = zkp_amd.bench_msm(pts, scal, g2=False, warmup=2, iters=iters, device=device)
    alt = zkp_amd.msm_g1(pts, scal, device=device, window_bits=13, table_depth=1)
    if alt != res:
        raise AssertionError("G1 MSM 2^20: bench result differs from the c=13/T=1 MSM of the same input")
    # each transform: the best of 3 runs of 20 back-to-back coset extensions (one run after the
    # proof loop is ~5 % slower than a cold one on the same box: clocks)
    ntt_ms = min(zkp_amd.bench_ntt(log_n, warmup=3, iters=20, device=device) for _ in range(3))
    ntt23_ms = min(zkp_amd.bench_ntt(23, warmup=3, iters=20, device=device) for _ in range(3))
    # the batched extension of three vectors (every pass one launch over all three: the split
    # quotient stage runs this; the proof keeps one vector per launch, DESIGN.md §5 NTT), per vector
    b20 = min(zkp_amd.bench_ntt(log_n, warmup=3, iters=20, device=device, count=3) for _ in range(3)) / 3
    b23 = min(zkp_amd.bench_ntt(23, warmup=3, iters=20, device=device, count=3) for _ in range(3)) / 3
    return {
        "msm_kind": "fixed-base: T-row tables 2^(c t) P (t < T) precomputed once per point set, as the prover "
                    "builds them at zkey load (the Groth16 bases are fixed); their build time is "
                    "msm_g1_2^20_table_build_ms, outside msm_g1_2^20_ms",
        "msm_g1_2^20_ms": round(st["ms_per_msm"], 3),
        "msm_g1_2^20_table_build_ms": round(st["table_build_ms"], 3),
        "msm_g1_2^20_table_rows": st["table_depth"],
        "msm_g1_2^20_result_check": "equal to the c=13/T=1 MSM of the same input",
        "msm_g1_2^20_Mpts_per_s": round(n / st["ms_per_msm"] / 1e3, 1),
        "msm_g1_2^20_accumulate_ms": round(st["ms_accumulate"], 3),
        "msm_window_bits": st["c"],
        "ntt_fr_2^20_coset_extend_ms": round(ntt_ms, 3),
        "ntt_roofline": {"2^20": ntt_roofline(log_n, ntt_ms), "2^23 (Venmo domain)": ntt_roofline(23, ntt23_ms),
                         "2^20 batched x3, per vector": ntt_roofline(log_n, b20),
                         "2^23 batched x3, per vector": ntt_roofline(23, b23)},
    }, st, (pts, scal, res)


def ntt_roofline(log_n, ms):
    """Roofline of one coset extension (iNTT -> coset key g^i/n -> NTT) of 2^log_n
    Fr elements.  Algorithmic work: 2 * (n/2) * log2 n butterfly products + n key products, 136 MAC per Fr
    mul; algorithmic bytes: one read + one write of n x 32 B.  Four-step passes of <= 8
    bits: 2 * ceil(log_n / 8) - 1 HBM round trips (the innermost inverse/forward pair is fused)."""
    n = 1 << log_n
    peak, _ = load_peak()
    mac = (2 * (n // 2) * log_n + n) * MAC_PER_FPMUL
    achieved = mac / (ms * 1e-3) / 1e12
    passes = 2 * ((log_n + 7) // 8) - 1
    out = {"bound": "valu-int", "ms": round(ms, 4), "achieved": round(achieved, 3), "peak": peak,
           "unit": "TMAC/s", "frac": round(achieved / peak, 4) if peak else None,
           "frac_vs_issue_ceiling": round(achieved / ISSUE_CEILING_TOPS, 4),
           "hbm_pass_GBps": round(passes * 64 * n / (ms * 1e-3) / 1e9, 1),
           "hbm_frac_of_8TBps": round(passes * 64 * n / (ms * 1e-3) / 8e12, 4)}
    cnt = load_ntt_issue().get("2^%d" % log_n)
    if cnt:  # counted on the same library (profiles/ntt_issue_r05.json): per-kernel issue at its own clock
        out["valu_lane_instr_per_element_pmc"] = cnt["coset_extension_valu_lane_instr_per_element"]
        out["valu_issue_frac_pmc"] = {k: v["valu_issue_frac"] for k, v in cnt["kernels"].items()}
        out["clock_GHz_pmc"] = {k: v["clock_GHz"] for k, v in cnt["kernels"].items()}
        out["pmc_source"] = "profiles/ntt_issue_r05.json"
    return out


S24 = dict(n_vars=16_000_000, n_constraints=(1 << 24) - 27, n_public=26)  # configs[4]


def run_split(args, rank, world, local):
    """configs[4]: ONE proof of the synthetic 2^24-constraint circuit split by point range
    over `world` GPUs (torchrun, backend nccl = RCCL: the partials are all-gathered over
    xGMI) or, in one process, over --parts slices on one GPU (emulation: the slices run
    one after another; reports the per-slice time and checks the combined proof against
    the unsplit proof bit-exactly)."""
    import torch
    if args.quotient == "dist":
        # the quotient-vector owners (parts 0..2) take fewer points (prover.hip split_range; every
        # rank and the slice exchange read the same setting): S24 over 8 slices 13.3 -> 9.7 ms
        os.environ.setdefault("ZKP_SPLIT_BALANCE", "1")
    scale = args.scale
    circ = synth.Circuit(int(S24["n_vars"] * scale), int(S24["n_constraints"] * scale), S24["n_public"], CIRCUIT_SEED)
    t0 = time.time()
    wit = circ.witness(1)
    zk = circ.zkey(SETUP_SEED, device=local)
    log("[rank %d] S24 circuit + witness + zkey (%.2f GB): %.1fs" % (rank, zk.len / 1e9, time.time() - t0))
    R_FIX, S_FIX = 0x1234567, 0x7654321
    if world > 1:
        import torch.distributed as dist
        from zkp_amd.dist import SplitProver
        sp = SplitProver(zk, local)
        sp.prover.stage(wit, slot=0)
        distq = args.quotient == "dist"

        def one():
            if distq:
                return sp.prove_raw_distq(wit, R_FIX, S_FIX, slot=0, staged=True)
            return sp.prove_raw(wit, R_FIX, S_FIX, staged_slot=0)
        for _ in range(args.warmup):
            one()
        dist.barrier()
        torch.cuda.synchronize(local)
        t_start = time.perf_counter()
        for _ in range(args.steps):
            res = one()
        torch.cuda.synchronize(local)
        el = torch.tensor([time.perf_counter() - t_start], dtype=torch.float64, device="cuda:%d" % local)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
        parts_desc = "%d ranks, RCCL all-gather of %d-byte partials, quotient %s" % (
            world, zkp_amd.PARTIAL_BYTES,
            "distributed (rank v%%G extends vector v, RCCL send/recv of domain slices)" if distq
            else "recomputed on every rank")
        check = None
    else:
        from zkp_amd.dist import split_range
        nparts = args.parts
        provers = [zkp_amd.Prover(zk, devices=[local], part=k, nparts=nparts) for k in range(nparts)]
        for p in provers:
            p.stage(wit, slot=0)
        distq = args.quotient == "dist"
        n = provers[0].domain_size
        full = [torch.empty(n * 32, dtype=torch.uint8, device="cuda:%d" % local) for _ in range(3)] if distq else None

        def one(per):
            parts = []
            if distq:  # rank k's work = its quotient vectors + its slice; the exchange is a device copy here
                for k, p in enumerate(provers):
                    mine = [v for v in range(3) if v % nparts == k]
                    t1 = time.perf_counter()
                    if mine:
                        p.quotient_part_staged(0, sum(1 << v for v in mine),
                                               [full[v].data_ptr() if v in mine else None for v in range(3)])
                    per[k] += time.perf_counter() - t1
                for k, p in enumerate(provers):
                    lo, hi = split_range(n, k, nparts)
                    sl = [full[v][lo * 32:hi * 32].clone() for v in range(3)]
                    torch.cuda.synchronize(local)
                    t1 = time.perf_counter()
                    parts.append(p.prove_partial_ext_staged(0, [t.data_ptr() for t in sl]))
                    per[k] += time.perf_counter() - t1
            else:
                for k, p in enumerate(provers):
                    t1 = time.perf_counter()
                    parts.append(p.prove_partial_staged(0))
                    per[k] += time.perf_counter() - t1
            return parts
        for _ in range(args.warmup):
            one([0.0] * nparts)
        per = [0.0] * nparts
        t_start = time.perf_counter()
        for _ in range(args.steps):
            res = zkp_amd.proof_combine_raw(zk, one(per), wit, R_FIX, S_FIX)
        elapsed = time.perf_counter() - t_start
        parts_desc = "%d slices emulated one after another on 1 GPU, quotient %s%s; per-slice ms %s" % (
            nparts, "distributed" if distq else "recomputed per slice",
            ", balanced point slices (ZKP_SPLIT_BALANCE=1)" if os.environ.get("ZKP_SPLIT_BALANCE") == "1" else "",
            [round(x / args.steps * 1e3, 2) for x in per])
        del provers
        full = zkp_amd.Prover(zk, devices=[local])
        check = full.prove_raw(wit, R_FIX, S_FIX) == res
        del full
    if rank != 0:
        return
    out = {
        "metric": "Groth16 proofs/sec (node) + 1-proof latency; configs[4] single proof split by point range",
        "value": round(args.steps / elapsed, 4), "unit": "proofs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32-limb Fp/Fr (BN254 integer arithmetic)",
        "data": "synthetic 2^24-constraint circuit, insecure known-tau zkey",
        "config": {"workload": "configs[4]: one proof split by point range", "n_vars": circ.n_vars,
                   "n_constraints": circ.n_constraints, "domain": circ.domain_size, "split": parts_desc},
        "bit_exact_vs_unsplit": check,
    }
    print(json.dumps(out), flush=True)


def batch_pcie_inclusive(args, circ, prover, wit, refs, rank, world, ndev, dist, sync, r_fix, s_fix):
    """configs[3] with the witness upload included: args.batch proofs per rank through
    zkp_prove_batch from HOST memory over all of this process's devices (args.batch_distinct
    distinct witnesses cycled; every proof copies its witness over PCIe), two workers per
    pipeline so the next witness's H2D overlaps the current proof.  One warm-up call first.
    Every batch proof is compared with a separately computed proof of the same witness (the
    staged reference proofs, or one zkp_prove per extra witness before the timed region).
    Whole-job proofs/s (max over ranks), for comparison with the staged headline."""
    k = max(1, args.batch_distinct)
    extra = gen_witnesses(circ, [500000 + 1000 * rank + i for i in range(max(0, k - len(wit)))])
    host = (list(wit) + extra)[:k]
    ref = list(refs[:len(host)]) + [prover.prove_raw(w, r_fix, s_fix) for w in host[len(refs):]]
    order = [i % k for i in range(args.batch)]
    # untimed warm-up batch: two proofs per worker (2 workers x ZKP_INFLIGHT pipelines x devices), so
    # every pipeline, upload slot and encode thread has run before the timed batch
    nwarm = 2 * 2 * int(os.environ.get("ZKP_INFLIGHT", "1")) * ndev
    prover.prove_batch_raw([host[i % k] for i in range(nwarm)], [r_fix] * nwarm, [s_fix] * nwarm)
    if dist:
        dist.barrier()
    sync()
    quiesce_gc()
    rx = roctx()  # a "batch timed" range for a profiler (tools/prof/batch_gaps.py)
    if rx:
        rx.roctxRangePushA(b"batch timed")
    t0 = time.perf_counter()
    res = prover.prove_batch_raw([host[i] for i in order], [r_fix] * len(order), [s_fix] * len(order))
    sync()
    el = time.perf_counter() - t0
    if rx:
        rx.roctxRangePop()
    if dist:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    bad = [j for j in range(len(order)) if j >= len(res) or res[j] != ref[order[j]]]
    vmode = prover.verify_mode()
    return {"proofs_per_rank": len(order), "distinct_host_witnesses": k, "n_gpus": world * ndev,
            "verify_before_return_mode": vmode,
            "verified": "%d/%d" % (len(res) if vmode != 0 else 0, len(order)),
            "proofs_per_s": round(len(order) * world / el, 3), "ms_per_proof": round(el / len(order) * 1e3, 3),
            "all_proofs_ok": len(res) == len(order) and not bad, "mismatched_proofs": bad[:8],
            "check": "every batch proof == a separately computed proof of the same witness at the same r, s",
            "pipelines_per_device": int(os.environ.get("ZKP_INFLIGHT", "1")),
            "workers_per_pipeline": 2,
            "note": "zkp_prove_batch from pageable host memory over %d device(s): the compact transfer of "
                    "witness i+1 (16 encode threads, pinned staging, 4 copy queues) runs while proof i computes"
                    % ndev}


def quiesce_gc():
    """Collect, then move every live Python object to the permanent generation (gc.freeze) before a
    timed region.  The harness holds millions of long-lived objects (synthetic circuit, witnesses,
    reference proofs); a full collection triggered by the batch binding's few hundred result objects
    walks all of them and stalled a 256-proof batch for 215-260 ms before its first or after its last
    kernel (profiles/batch_gc_r05.txt) -- a harness artefact, not the prover's (the C ABI allocates no
    Python objects)."""
    gc.collect()
    gc.freeze()


def roctx():
    """The ROCTx marker library, if present (marks the timed region for a profiler; no-op otherwise)."""
    for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"):
        try:
            return ctypes.CDLL(os.path.join("/opt/rocm/lib", name))
        except OSError:
            pass
    return None


def accumulate_rooflines(launches, peak, peak_src, traffic):
    """Per-launch roofline of the bucket-accumulate kernels (HIP events around every timed launch,
    zkp_prover_launch_stats).  The headline `roofline` is the H MSM's launch, which runs with the
    GPU mostly to itself at the end of the proof; the witness launches (A, B1, C: beside the quotient
    and the other streams) and the G2 launch (B2) are reported per launch kind.  Algorithmic work per
    mixed addition: G1 11 Fp-mul x 136 MAC, G2 3x that (Fq2)."""
    kinds = {}
    for r in launches:
        kinds.setdefault(r["msm"], []).append(r)

    def line(rs, mult, kernel):
        adds = sum(r["adds"] for r in rs) / len(rs)
        ms = sum(r["ms"] for r in rs) / len(rs)
        mac = adds * FPMUL_PER_MADD * MAC_PER_FPMUL * mult
        ach = mac / (ms * 1e-3) / 1e12 if ms > 0 else None
        return {"kernel": kernel, "launches": len(rs), "mixed_adds_per_launch": int(adds),
                "workgroups": sorted(set(r["blocks"] for r in rs)),
                "avg_launch_ms": round(ms, 4), "ms_min": round(min(r["ms"] for r in rs), 4),
                "ms_max": round(max(r["ms"] for r in rs), 4),
                "achieved": round(ach, 3) if ach else None, "frac": round(ach / peak, 4) if (ach and peak) else None}
    lines = {}
    for k in ("A", "B1", "C", "H"):
        if k in kinds:
            lines[k] = line(kinds[k], 1, "k_accumulate<Fq>")
    if "B2" in kinds:
        lines["B2"] = line(kinds["B2"], 3, "k_accumulate<Fq2>")
    pk = (traffic or {}).get("per_kind", {})
    busy = load_valu_counted()
    for k, ln in lines.items():  # counted issue share and clock of the same kernel (each launch alone)
        kk = "H" if k == "H" else ("B2" if k == "B2" else "witness (A, B1, C)")
        src = pk.get(kk)
        if src:
            ln.update(src)
        if kk in busy:
            ln["valu_busy_counted_pmc"] = busy[kk]
        if ln.get("achieved"):
            ln["frac_vs_issue_ceiling"] = round(ln["achieved"] / ISSUE_CEILING_TOPS, 4)
    h = lines.get("H") or {}
    roofline = {
        "kernel": "k_accumulate<Fq>, the H MSM launch (G1 bucket accumulation, XYZZ mixed adds)",
        "bound": "valu-int",
        "achieved": h.get("achieved"),
        "peak": peak,
        "unit": "TMAC/s (32x32->64 v_mad_u64_u32)",
        "frac": h.get("frac"),
        "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
        "traffic_source": traffic.get("source") if traffic else None,
        "algorithmic_work_per_launch": {"mixed_adds": h.get("mixed_adds_per_launch"), "fp_mul_per_add": FPMUL_PER_MADD,
                                        "mac_per_fp_mul": MAC_PER_FPMUL},
        "valu_issue_frac_pmc": traffic.get("valu_issue_frac") if traffic else None,
        "valu_busy_counted_pmc": busy.get("H"),
        "valu_busy_note": "valu_issue_frac_pmc prices every VALU instruction at one quad-cycle; valu_busy_counted_pmc "
                          "subtracts the quad-cycles two waves' full-rate instructions shared (SQ_ACTIVE_INST_VALU2, "
                          "profiles/pmc_valu_r06.json): 1.6 % of the H launch's instructions",
        "clock_GHz_pmc": traffic.get("clock_GHz") if traffic else None,
        "frac_vs_issue_ceiling": round(h["achieved"] / ISSUE_CEILING_TOPS, 4) if h.get("achieved") else None,
        "issue_ceiling": ISSUE_CEILING_TOPS,
        "issue_ceiling_note": "one v_mad_u64_u32 per SIMD per quad-cycle (4 clocks, profiles/valu_rates_r06.txt) on "
                              "1024 SIMDs at 2.4 GHz; full-rate 2-clock ops gain only when two waves co-issue them",
        "traffic_note": "HBM bytes per launch (FETCH x1 + WRITE): ~101 B per mixed addition, 1.49x the per-addition "
                        "minimum (64-B base + 4-B index = 68 B) and 13.7x SURVEY.md §8d's MSM floor (2^23 x 96 B): the "
                        "cost of the 13-row precomputed base table (random gathers over 7 GB; 2.6 L1-TLB misses per "
                        "addition), at ~1.4 TB/s, 18 % of HBM",
        "valu_lane_instructions_per_addition_pmc": traffic.get("valu_lane_instructions_per_addition") if traffic else None,
        "avg_launch_ms": h.get("avg_launch_ms"),
        "launches_timed": h.get("launches"),
        "peak_source": peak_src,
        "note": "integer-multiply (VALU) bound, no MFMA/HBM bound applies (SURVEY.md §8d D3); frac counts the "
                "algorithmic 136 MAC per Fp mul; per-launch-kind lines in roofline_launches (A, B1, C, B2 share "
                "the GPU with the quotient and the other streams)",
    }
    if traffic and h.get("avg_launch_ms"):
        # traffic is the PMC average over all G1 launches; reported against the H launch time
        roofline["hbm_GBps"] = round(traffic["hbm_bytes_per_launch"] / (h["avg_launch_ms"] * 1e-3) / 1e9, 1)
    g2 = lines.get("B2")
    roofline_g2 = None
    if g2:
        roofline_g2 = dict(g2, bound="valu-int", peak=peak, unit="TMAC/s (32x32->64 v_mad_u64_u32)",
                           work="3 x the G1 unit per Fq2 mixed addition (SURVEY.md §8d D4)")
    return roofline, {"per_kind": lines, "roofline_g2": roofline_g2}


def bool0_line(args, device, r_fix, s_fix, steps=4):
    """The bound of the witness assumption: the Venmo-shaped circuit with every defined signal uniform
    (bool_pct 0: the witness MSMs then carry ~W digits per signal instead of ~1.6), its own key, staged
    witnesses, on a prover of its own (the caller releases the headline prover first)."""
    c0 = synth.Circuit.venmo(CIRCUIT_SEED, bool_pct=0)
    ws = gen_witnesses(c0, [900001 + i for i in range(2)])
    zk = c0.zkey(SETUP_SEED, device=device)
    p = zkp_amd.Prover(zk, devices=[device])
    for i, w in enumerate(ws):
        p.stage(w, slot=i)
    p.prove_staged_raw(0, r_fix, s_fix)
    ref = [p.prove_raw(w, r_fix, s_fix) for w in ws]
    t0 = time.perf_counter()
    res = [p.prove_staged_raw(i % 2, r_fix, s_fix) for i in range(steps)]
    el = time.perf_counter() - t0
    ok = all(r == ref[i % 2] for i, r in enumerate(res))
    p.close()
    return {"witness_bool_pct": 0, "proofs_per_s": round(steps / el, 3), "ms_per_proof": round(el / steps * 1e3, 3),
            "steps": steps, "all_proofs_ok": ok,
            "note": "Venmo shape, every defined signal uniform (its own key; the worst case of the witness "
                    "MSMs); the headline assumes 70 % bit-valued signals"}


def cpu_baseline(args, zk, wit0, gpu_proof, r_fix, s_fix, msm_case):
    """The CPU column: snarkjs / rapidsnark are not in this image, so the
    build's own multithreaded C++ restatement (oracle/cpu, "build CPU restatement, not
    snarkjs") proves the same zkey/witness 0 on every usable host core; its G1 MSM times
    the configs[1] 2^20 MSM.  Both results are compared with the GPU's.  Published
    reference numbers (other hardware) ride along, labelled."""
    info = host_cpu_info()
    threads = args.cpu_threads or info["usable_cores"]
    try:
        from oracle import cpu_oracle
        t0 = time.time()
        (ca, cb, cc), cms = cpu_oracle.prove(None, wit0, r_fix, s_fix, threads=threads, zkey_ptr=zk.ptr,
                                              zkey_len=zk.len)
        cpu_s = time.time() - t0
        res = {
            "value": round(1.0 / cpu_s, 5), "unit": "proofs/s", "cores": threads, "kind": "port",
            "label": "build CPU restatement, not snarkjs",
            "sample": "one full Venmo-shaped proof (same zkey/witness 0) by the oracle/cpu C++ restatement on "
                      "%d threads: %.1f s (abc %.0f, ntt %.0f, g1 %.0f, g2 %.0f ms)" % (
                          threads, cpu_s, cms[0], cms[1], cms[2], cms[3]),
            "bit_exact_vs_gpu": (ca, cb, cc) == gpu_proof,
            "host": info,
            "published": PUBLISHED_CPU,
        }
        if msm_case is not None:
            pts, scal, gres = msm_case
            t0 = time.time()
            cres = cpu_oracle.msm_g1(pts, scal, threads=threads)
            ms = (time.time() - t0) * 1e3
            res["msm_g1_2^20"] = {"ms": round(ms, 1), "Mpts_per_s": round((len(scal) // 32) / ms / 1e3, 2),
                                  "bit_exact_vs_gpu": cres == gres}
        return res
    except Exception as e:  # reported, never silently replaced
        return {"value": None, "error": str(e), "host": info, "published": PUBLISHED_CPU}


def sustained_line(args, prover, ndev, nw, refs, dist, sync, on_devices, r_fix, s_fix):
    """The staged headline loop run for >= args.sustain_s seconds: one proof at a time
    per device, every proof compared with the reference proof of its witness.  The 20-step headline is a
    ~0.5-s window on a chip that runs power-limited (1.8-2.3 GHz under these kernels); this
    is the node-throughput figure over ~1,250 proofs."""
    counts = [0] * ndev
    bad = []
    stop = [False]

    def loop(d):
        i = 0
        while not stop[0]:
            pr = prover.prove_staged_raw(i % nw, r_fix, s_fix, dev_index=d)
            if pr != refs[i % nw]:
                bad.append((d, i))
            i += 1
            counts[d] = i
    # proofs per window of ~sustain_s / 10 (at most 30 s), printed to stderr as it goes: a long run shows
    # progress, and the windows show whether the rate drifts (clock, heat) over the run
    wlen = min(30.0, max(1.0, args.sustain_s / 10))
    windows = []

    def monitor():
        last_n, last_t = 0, time.perf_counter()
        while not stop[0]:
            time.sleep(0.25)
            now = time.perf_counter()
            if now - last_t >= wlen and not stop[0]:
                n_now = sum(counts)
                windows.append(round((n_now - last_n) / (now - last_t), 2))
                print("sustain: %.0f s, %d proofs, %.2f proofs/s in the last window"
                      % (now - t0, n_now, windows[-1]), file=sys.stderr, flush=True)
                last_n, last_t = n_now, now
    if dist:
        dist.barrier()
    sync()
    quiesce_gc()
    timer = threading.Timer(args.sustain_s, lambda: stop.__setitem__(0, True))
    t0 = time.perf_counter()
    timer.start()
    mon = threading.Thread(target=monitor, daemon=True)
    mon.start()
    on_devices(loop)
    sync()
    el = time.perf_counter() - t0
    timer.cancel()
    stop[0] = True
    mon.join()
    n = sum(counts)
    if dist:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        t = torch.tensor([float(n)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        n = int(t.item())
    return {"proofs_per_s": round(n / el, 3), "proofs": n, "seconds": round(el, 2),
            "ms_per_proof": round(el / max(1, n) * 1e3 * ndev, 3), "all_proofs_ok": not bad,
            "mismatched_proofs": bad[:8], "window_s": wlen, "window_proofs_per_s": windows,
            "note": "staged loop, one proof at a time per device, for >= %.0f s; every proof checked" % args.sustain_s}


def compact_line(out):
    """The contract line the driver keeps (its record holds the last 8 KB of stdout):
    the metric's two halves (proofs/s and 1-proof latency), the sustained and batch rates, the headline
    roofline and cpu_baseline, and the configs[1] kernel numbers.  Everything else is in the
    {"bench_detail": ...} line printed just before it."""
    keep = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "latency_ms", "latency_ms_staged",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "value_note", "all_proofs_ok",
            "rehearsal"]
    c = {k: out[k] for k in keep if k in out}
    cfg = out.get("config", {})
    c["config"] = {k: cfg[k] for k in ("workload", "n_vars", "n_constraints", "n_public", "domain",
                                      "witness_bool_pct", "parallelism") if k in cfg}
    su = out.get("sustained")
    if su:
        c["sustained"] = {k: su.get(k) for k in ("proofs_per_s", "proofs", "seconds", "vs_value", "all_proofs_ok")}
    b = out.get("batch_pcie_inclusive")
    if b:
        c["batch_pcie_inclusive"] = {k: b.get(k) for k in ("proofs_per_s", "proofs_per_rank", "verified",
                                                          "vs_staged_headline", "all_proofs_ok")}
    two = out.get("staged_two_in_flight")
    if two:
        c["staged_two_in_flight_proofs_per_s"] = two.get("proofs_per_s")
    r = out.get("roofline") or {}
    c["roofline"] = {k: r[k] for k in ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic",
                                      "algorithmic_work_per_launch", "avg_launch_ms", "launches_timed",
                                      "valu_issue_frac_pmc", "valu_busy_counted_pmc", "clock_GHz_pmc",
                                      "frac_vs_issue_ceiling", "issue_ceiling", "hbm_GBps", "peak_source")
                     if k in r}
    g2 = (out.get("roofline_launches") or {}).get("roofline_g2")
    if g2:
        c["roofline_g2_frac"] = g2.get("frac")
    cb = out.get("cpu_baseline")
    if cb:
        c["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "label", "sample",
                                                   "bit_exact_vs_gpu", "error") if k in cb}
    au = out.get("all_uniform_witness")
    if au:
        c["all_uniform_witness"] = {k: au.get(k) for k in ("proofs_per_s", "ms_per_proof", "all_proofs_ok")}
    kb = out.get("kernels_config1")
    if kb:
        nr = kb.get("ntt_roofline", {})
        c["kernels_config1"] = {
            "msm_g1_2^20_Mpts_per_s": kb.get("msm_g1_2^20_Mpts_per_s"), "msm_g1_2^20_ms": kb.get("msm_g1_2^20_ms"),
            "msm_kind": "fixed-base (table build %s ms, outside)" % kb.get("msm_g1_2^20_table_build_ms"),
            "ntt_2^20_ms": (nr.get("2^20") or {}).get("ms"), "ntt_2^20_frac": (nr.get("2^20") or {}).get("frac"),
            "ntt_2^23_ms": (nr.get("2^23 (Venmo domain)") or {}).get("ms"),
            "ntt_2^23_frac": (nr.get("2^23 (Venmo domain)") or {}).get("frac")}
    c["detail"] = "the {\"bench_detail\": ...} stdout line before this one (per-launch rooflines, stage ms, PMC)"
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--witnesses", type=int, default=4, help="distinct staged witnesses per rank (cycled)")
    ap.add_argument("--cpu-baseline", choices=["full", "none"], default="full")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable host core (nproc, cgroup quota)")
    ap.add_argument("--no-kernels", action="store_true")
    ap.add_argument("--batch", type=int, default=256,
                    help="configs[3] PCIe-inclusive batch line: proofs per rank from HOST witnesses via "
                         "zkp_prove_batch (0 = skip); reported beside the staged headline, never as `value`")
    ap.add_argument("--batch-distinct", type=int, default=16, help="distinct host witnesses cycled by the batch")
    ap.add_argument("--bool-pct", type=int, default=70,
                    help="witness mix: percent of bit-valued (AND/XOR) signals; 70 = the default assumption, "
                         "0 = all-uniform witness (sensitivity of the witness MSMs to the real witness)")
    ap.add_argument("--no-bool0-line", dest="bool0_line", action="store_false",
                    help="skip the all-uniform-witness sub-line (the bound of the witness assumption)")
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the Venmo shape (smoke/debug only)")
    ap.add_argument("--quotient", choices=["dist", "full"], default="dist",
                    help="split mode: distribute the three coset extensions over the ranks, or recompute per rank")
    ap.add_argument("--mode", choices=["replicas", "split"], default="replicas",
                    help="replicas: independent proofs per GPU (headline); split: configs[4], one proof over GPUs")
    ap.add_argument("--parts", type=int, default=2, help="split mode in one process: slices on one GPU")
    ap.add_argument("--inflight", type=int, default=1,
                    help="staged proofs in flight per device in the timed loop (host threads per device, up to "
                         "ZKP_INFLIGHT pipelines).  1 (default) keeps every accumulate launch's time its own (the "
                         "per-launch rooflines); the line also reports 2 in flight as staged_two_in_flight")
    ap.add_argument("--sustain-s", type=float, default=30.0,
                    help="seconds of the sustained staged loop reported beside the 20-step headline (0 = skip)")
    ap.add_argument("--detail-out", default="",
                    help="also write the detailed JSON object to this file (it is always printed as an earlier "
                         "stdout line {\"bench_detail\": ...}; the last line is the compact contract line)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="--gpus N without torchrun on fewer GPUs: N logical devices on one GPU (code-path check; "
                         "the line says \"rehearsal\": true and is not a scaling number)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("ZKP_BENCH_DEVICE"):  # rehearsal only: put every rank on one GPU
        local = int(os.environ["ZKP_BENCH_DEVICE"])
    dist = None
    if args.mode == "split":
        if world > 1:
            import torch
            import torch.distributed as tdist
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl")  # RCCL: the partial-sum all-gather runs over xGMI
        return run_split(args, rank, world, local)
    if world > 1:
        if args.gpus not in (1, world):
            log("bench.py: --gpus %d but torchrun started %d ranks (one GPU per rank)" % (args.gpus, world))
            sys.exit(2)
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")  # measurement plumbing only (barrier / max); the path has no collective
        devices, rehearsal = [local], False
    else:
        # one process driving N devices (one host process, a resident key per GPU)
        if args.gpus < 1:
            log("bench.py: --gpus must be >= 1")
            sys.exit(2)
        rehearsal = args.rehearsal and args.gpus > 1
        if rehearsal:
            devices = [local] * args.gpus
        else:
            visible = visible_devices()
            if visible < args.gpus:
                log("bench.py: --gpus %d requested but only %d GPU(s) visible; refusing to report a %d-GPU "
                    "number from fewer devices (use --rehearsal to map %d logical devices onto device %d)"
                    % (args.gpus, visible, args.gpus, args.gpus, local))
                sys.exit(2)
            devices = list(range(args.gpus)) if args.gpus > 1 else [local]
    ndev = len(devices)

    t_setup = time.time()
    if args.scale == 1.0:
        circ = synth.Circuit.venmo(CIRCUIT_SEED, bool_pct=args.bool_pct)
    else:
        v = synth.VENMO
        circ = synth.Circuit(int(v["n_vars"] * args.scale), int(v["n_constraints"] * args.scale), v["n_public"],
                             CIRCUIT_SEED, bool_pct=args.bool_pct)
    nw = max(1, min(args.witnesses, args.steps + args.warmup))
    wseeds = [1000 * rank + i + 1 for i in range(nw)]
    wit = gen_witnesses(circ, wseeds)
    log("[rank %d] circuit + %d witnesses: %.1fs" % (rank, nw, time.time() - t_setup))
    t0 = time.time()
    # host threads for the synthetic key's QAP evaluation: share the host between the ranks
    zk = circ.zkey(SETUP_SEED, device=devices[0], threads=max(1, (os.cpu_count() or 8) // max(1, world)))
    log("[rank %d] synthetic zkey (%.2f GB): %.1fs" % (rank, zk.len / 1e9, time.time() - t0))
    t0 = time.time()
    # two pipelines per device sharing the base tables: the batch line keeps two proofs in
    # flight per GPU (+2.4% measured, profiles/inflight_r02.txt); the staged headline runs on
    # each device's first pipeline
    # (a rehearsal maps N logical devices onto one GPU: one pipeline each, or 2N pipelines would share
    # one GPU's HBM)
    os.environ.setdefault("ZKP_INFLIGHT", "1" if rehearsal else "2")
    prover = zkp_amd.Prover(zk, devices=devices)
    for d in range(ndev):
        for i, w in enumerate(wit):
            prover.stage(w, slot=i, dev_index=d)
    log("[rank %d] zkey resident in HBM of %d device(s) %s + witnesses staged: %.1fs"
        % (rank, ndev, devices, time.time() - t0))

    R_FIX, S_FIX = 0x1234567, 0x7654321

    def on_devices(fn):
        """fn(d) for every device index, concurrently (one host thread per device)."""
        if ndev == 1:
            fn(0)
            return
        errs = []

        def run(d):
            try:
                fn(d)
            except BaseException as e:  # re-raised below
                errs.append(e)
        ths = [threading.Thread(target=run, args=(d,)) for d in range(ndev)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]

    on_devices(lambda d: [prover.prove_staged_raw(i % nw, R_FIX, S_FIX, dev_index=d) for i in range(args.warmup)])
    # reference proofs of the staged witnesses (device 0), computed before the timed region
    refs = [prover.prove_staged_raw(i, R_FIX, S_FIX, dev_index=0) for i in range(nw)]
    prover.instrument(True)

    def sync():
        try:
            import torch
            if torch.cuda.is_available():
                for d in sorted(set(devices)):
                    torch.cuda.synchronize(d)
        except Exception:
            pass

    if dist:
        dist.barrier()
    sync()
    per_dev = [None] * ndev

    inflight = max(1, args.inflight)

    def timed(d, inflight=inflight):
        # `inflight` host threads per device, proof i on thread i % inflight: each staged call takes an
        # idle pipeline of the device (Prover::prove_staged), so that many proofs are in flight
        out = [None] * args.steps
        if inflight <= 1:
            out[:] = [prover.prove_staged_raw(i % nw, R_FIX, S_FIX, dev_index=d) for i in range(args.steps)]
        else:
            errs = []

            def lane(t):
                try:
                    for i in range(t, args.steps, inflight):
                        out[i] = prover.prove_staged_raw(i % nw, R_FIX, S_FIX, dev_index=d)
                except BaseException as e:  # re-raised below
                    errs.append(e)
            ths = [threading.Thread(target=lane, args=(t,)) for t in range(inflight)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            if errs:
                raise errs[0]
        per_dev[d] = out
    quiesce_gc()
    rx = roctx()  # a "bench timed" range in a rocprofv3 --marker-trace (tools/prof/launch_split.py)
    if rx:
        rx.roctxRangePushA(b"bench timed")
    t_start = time.perf_counter()
    on_devices(timed)
    sync()
    elapsed = time.perf_counter() - t_start
    if rx:
        rx.roctxRangePop()
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    results = per_dev[0]
    mismatch = [(d, i) for d in range(ndev) for i in range(args.steps) if per_dev[d][i] != refs[i % nw]]
    kstats = prover.kernel_stats()
    msm_cfg = prover.msm_config()
    stage_ms = prover.timings()

    launches = prover.launch_stats()
    prover.instrument(False)
    # the same staged loop with two proofs in flight per device (the next proof's first kernels fill the
    # previous one's finishing tail: +1.3-2.2 % in round 3, profiles/inflight_hwq_r03.txt), every proof
    # checked; reported beside the headline, not as `value` (its launches overlap: no per-launch time)
    two = None
    if int(os.environ.get("ZKP_INFLIGHT", "1")) >= 2 and inflight == 1:
        if dist:
            dist.barrier()
        sync()
        t2 = time.perf_counter()
        on_devices(lambda d: timed(d, 2))
        sync()
        el2 = time.perf_counter() - t2
        bad2 = [(d, i) for d in range(ndev) for i in range(args.steps) if per_dev[d][i] != refs[i % nw]]
        two = {"proofs_per_s": round(args.steps * ndev / el2, 4), "ms_per_proof": round(el2 / args.steps * 1e3, 3),
               "all_proofs_ok": not bad2, "in_flight_per_device": 2}
        mismatch += [("two in flight", d, i) for d, i in bad2]
    # 1-proof latency, witness in HBM: one staged proof at a time (median of 5)
    lat_st = []
    for i in range(5):
        t0 = time.perf_counter()
        prover.prove_staged_raw(i % nw, R_FIX, S_FIX, dev_index=0)
        lat_st.append((time.perf_counter() - t0) * 1e3)
    staged_latency_ms = sorted(lat_st)[2]
    # 1-proof latency from a HOST witness (the reference call: zkp.ts:94, 5_gen_proof.sh:8): upload
    # through the pinned slot + proof + assembly, one proof at a time (median of 5, each checked)
    lat, up_ms, up_mb = [], [], []
    for i in range(5):
        t0 = time.perf_counter()
        pr = prover.prove_raw(wit[i % nw], R_FIX, S_FIX)
        lat.append((time.perf_counter() - t0) * 1e3)
        tm = prover.timings()
        up_ms.append(tm["wtns_h2d"])
        up_mb.append(tm["wtns_pcie_mb"])
        if pr != refs[i % nw]:
            mismatch.append(("host-witness latency proof", i))
    first_host_ms = lat[0]  # the process's first host-witness proof (upload slot 0 exists from load on)
    lat.sort()
    up_ms.sort()
    pcie_latency_ms, upload_ms = lat[len(lat) // 2], up_ms[len(up_ms) // 2]

    batch = None
    if args.batch > 0:
        batch = batch_pcie_inclusive(args, circ, prover, wit, refs, rank, world, ndev, dist, sync, R_FIX, S_FIX)

    sustained = None
    if args.sustain_s > 0:
        sustained = sustained_line(args, prover, ndev, nw, refs, dist, sync, on_devices, R_FIX, S_FIX)

    if rank != 0:
        return

    n_total = args.steps * world * ndev
    value = n_total / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    peak, peak_src = load_peak()
    traffic = load_traffic()
    roofline, acc_lines = accumulate_rooflines(launches, peak, peak_src, traffic)
    wit_bytes = circ.n_vars * 32

    out = {
        "metric": "Groth16 proofs/sec (node) + 1-proof latency, Venmo circuit; G1 MSM Mpts/s",
        "value": round(value, 4),
        "unit": "proofs/s",
        "n_gpus": world * ndev,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "latency_ms": round(pcie_latency_ms, 3),
        "latency_ms_staged": round(staged_latency_ms, 3),
        "latency_ms_first_host_proof": round(first_host_ms, 3),
        "staged_in_flight_per_device": inflight,
        "staged_two_in_flight": two,
        "latency_note": "latency_ms = one proof from a host witness (pinned-slot upload + proof + assembly), "
                        "median of 5; latency_ms_staged = one staged proof at a time (witness already in HBM), "
                        "median of 5; the timed loop keeps staged_in_flight_per_device proofs in flight per GPU",
        "witness_upload": {"ms": round(upload_ms, 3), "witness_bytes": wit_bytes,
                           "pcie_bytes": int(max(up_mb) * 1e6),
                           "witness_GBps": round(wit_bytes / (upload_ms * 1e-3) / 1e9, 1) if upload_ms > 0 else None,
                           "host_encode_threads": 16,
                           "note": "compact transfer: 16 host threads encode 64K-signal chunks (0/1 values as "
                                   "metadata bits, other values < 2^32 as one word) into pinned memory with "
                                   "non-temporal stores, each chunk's DMA on one of 4 copy queues as soon as it is "
                                   "encoded, one kernel expands them in HBM; ms = pageable witness -> 32-B layout "
                                   "in HBM"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32-limb Fp/Fr (BN254 integer arithmetic)",
        "data": "synthetic Venmo-shaped circuit + distinct synthetic witnesses, insecure known-tau zkey",
        "config": {"workload": "configs[2]: full Groth16 prove, Venmo-shaped circuit, 1 proof per step",
                   "n_vars": circ.n_vars, "n_constraints": circ.n_constraints, "n_public": circ.n_public,
                   "domain": circ.domain_size, "distinct_witnesses_per_rank": nw,
                   "witness_bool_pct": args.bool_pct,
                   "parallelism": "replicas%d" % (world * ndev),
                   "launch": "torchrun, one process per GPU" if world > 1 else
                             "one process, one resident prover over devices %s, one host thread per device" % devices,
                   "msm": msm_cfg},
        "all_proofs_ok": not mismatch,
        "proof_check": "every timed proof == the reference proof of the same staged witness (device 0, same r, s)",
        "stage_ms_last_proof": {k: round(v, 3) for k, v in stage_ms.items()},
        "batch_pcie_inclusive": batch,
        "sustained": sustained,
        "roofline": roofline,
        "roofline_launches": acc_lines,
    }

    if rehearsal:
        out["rehearsal"] = True
        out["rehearsal_note"] = ("%d logical devices mapped onto GPU %d (pipelines sharing one copy of the base "
                                 "tables): exercises the multi-device path; not a scaling measurement" % (ndev, local))
    if mismatch:
        out["mismatched_proofs"] = mismatch[:8]
    msm_case = None
    if batch:
        batch["vs_staged_headline"] = round(batch["proofs_per_s"] / value, 4)
    if not args.no_kernels:
        kb, kst, msm_case = kernel_benches(devices[0])
        out["kernels_config1"] = kb
        if peak and kst["ms_accumulate"] > 0:
            # the same kernel alone on the GPU (configs[1] G1 MSM 2^20, uniform scalars)
            iso = kst["mixed_adds"] * FPMUL_PER_MADD * MAC_PER_FPMUL / (kst["ms_accumulate"] * 1e-3) / 1e12
            roofline["isolated_launch"] = {"workload": "configs[1] G1 MSM 2^20 accumulate, kernel alone",
                                           "mixed_adds": kst["mixed_adds"], "avg_launch_ms": round(kst["ms_accumulate"], 4),
                                           "achieved": round(iso, 3), "frac": round(iso / peak, 4)}
    if args.bool0_line and args.bool_pct != 0 and args.scale == 1.0:
        prover.close()  # its HBM goes to the all-uniform line's prover
        out["all_uniform_witness"] = bool0_line(args, devices[0], R_FIX, S_FIX)

    if args.cpu_baseline == "full":
        out["cpu_baseline"] = cpu_baseline(args, zk, wit[0], results[0][0], R_FIX, S_FIX, msm_case)
    if sustained:
        sustained["vs_value"] = round(sustained["proofs_per_s"] / value, 4)
        if sustained["vs_value"] < 0.98:
            out["value_note"] = ("the %.0f-s sustained staged loop ran at %.4f of `value` (%.2f proofs/s): the chip "
                                 "runs power-limited under these kernels; node throughput over minutes is the "
                                 "sustained figure" % (sustained["seconds"], sustained["vs_value"],
                                                       sustained["proofs_per_s"]))
    print(json.dumps({"bench_detail": out}), flush=True)
    if args.detail_out:
        with open(args.detail_out, "w") as f:
            json.dump(out, f)
    print(json.dumps(compact_line(out)), flush=True)


if __name__ == "__main__":
    main()
