#!/usr/bin/env python3
"""Headline benchmark: minisched's scheduling cycle on MI355X.

Metric (BASELINE.json): pod x node filter+score evals/sec (and pods scheduled/sec)
at 100k nodes on 1/2/4/8 GPUs -> workload = config C: 100,000 nodes x
100,000 pods, NodeUnschedulable + NodeNumber, every (pod, node) pair evaluated
(K1 "pp", ms_sweep_pp.hip).

One step = the whole pod batch through the hot path with inputs resident in HBM:
  N = 1: ms_select_batch_device — ONE fused launch: filter -> score ->
         selectHost argmax -> decode of every pod (minisched.go:40-85).
  N > 1, --split nodes (default, the north star's node sharding): every rank's
         context joins one in-library RCCL communicator (sharded.init_comm) and
         a step is ms_sharded_submit: the sweep of all P pods against the
         rank's N/G-row shard, ONE grouped reduce-scatter (uint64 MAX of the
         packed keys) leaving each rank the combined keys of its P/G pods, and
         their decode — the library pipelines step k's collective under the
         next steps' sweeps; ms_sharded_drain ends the timed region. This is
         the path a Go scheduleOne binds.
  N > 1, --split pods: every rank holds the whole (100 KB) node table and runs
         the fused cycle on its P/G pods; no collective.
value = P * N / step time (max over ranks): whole-job evals/s.

Scaling (--scaling, default strong): config C as BASELINE.json states it —
100k nodes x 100k pods split over the N GPUs (each rank: 100k pods against its
100k/N rows, decode of its 100k/N pods). --scaling weak: every GPU brings its
own 100k-pod batch (N x 100k pods per step), a labelled extra.

Extra fields (rank 0): pods/s per SURVEY §8(d) — ms_schedule_batch_compact on
host arrays (8 B pods in, the cycle, bind commit, 8 B results out; single
shard: one launch over pinned host memory; 1 warm-up, median of 5; with N > 1
the collective host call over the communicator; `e2e`: ms_schedule_batch with
40/24 B records) — as the top-level `pods_per_s`, the device-resident rate as
`device_pods_per_s`, the VALU-issue roofline of the timed kernel with its HBM
figures, and the CPU baseline (oracle, OpenMP, on the box's host cores).

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 the driver
uses torch.distributed.run with one rank per GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))

METRIC = "pod×node filter+score evals/sec and pods scheduled/sec at 100k nodes, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_EVAL = {"NU+NN": 2, "NU+NRF+NN+LA": 58}
# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 integer VALU instruction per
# ~4 cycles per SIMD at 2.4 GHz = 614e9 wave-instructions/s (nominal); the
# measured ceiling of every instruction the kernel issues (bitop3, ffbl/ffbh,
# mad_u24, mul_lo, xor sdwa, max3) is 1.74-1.86 ns per wave-instruction per
# SIMD at 8 waves/SIMD (tools/ubench/valu_rates.hip, profiles/r02c_valu_rates.txt).
VALU_PEAK_NOMINAL = 256 * 4 * 2.4e9 / 4
VALU_PEAK_MEASURED = 256 * 4 / 1.75e-9
# MI355X_MICROARCH.md (lines 54, 473): a wave64 VALU op issues over 2 cycles on a
# SIMD-32, i.e. 1.229e12 wave-instructions/s chip-wide. No instruction reached it
# in our microbenchmark, packed controls included: at 1 / 2 / 4 / 8 / 16 waves per
# SIMD every one of 20 ops (v_bitop3, v_pk_fma_f32, v_pk_add_u16, v_max_f64, ...)
# converges to 4.1-4.2 cycles per wave-instruction per SIMD, and the counters say
# SQ_ACTIVE_INST_VALU = SQ_INSTS_VALU with 4.0 active cycles each
# (profiles/r05b_valu_issue.json), so `frac` stays against the 4-cycle rate and
# `frac_vs_guide_peak` reports the guide's figure beside it.
VALU_PEAK_GUIDE = 256 * 4 * 2.4e9 / 2
VALU_RATES_UBENCH = ("tools/ubench/valu_rates.hip + valu_pmc.sh -> profiles/r05b_valu_issue.json: 4.0 active "
                     "cycles per wave64 VALU instruction, 1-16 waves per SIMD, packed ops included")
PP_KERNEL = "k_sweep_nunn_pp"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # (N = 8: ~65 us a step; amortises pipeline fill and barriers)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C", choices=["B", "C", "D"])
    ap.add_argument("--split", default=None, choices=["nodes", "pods"],
                    help="N > 1 partition (default: nodes for B/C, pods for D)")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default): the config's P pods split over the GPUs (BASELINE config C); weak: "
                         "every GPU brings the config's pod batch, so the job schedules N x P pods")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the e2e measurements and configs B, D, E")
    ap.add_argument("--no-configs", action="store_true", help="skip configs B, D, E (device + CPU baselines)")
    ap.add_argument("--profile-json", default=os.path.join(ROOT, "profiles", "r06o_pmc_C.json"),
                    help="rocprofv3 counter summary of the timed kernel (tools/profile_pp.sh)")
    ap.add_argument("--profile-shard-prefix", default=os.path.join(ROOT, "profiles", "r04zh_pmc_shard"),
                    help="N > 1: per-shard K1 counters <prefix><rows>.json (tools/profile_shards.sh)")
    ap.add_argument("--profile-json-e", default=os.path.join(ROOT, "profiles", "r06ag_pmc_E.json"),
                    help="rocprofv3 counter summary of config E's step kernel (tools/profile_e.sh)")
    return ap.parse_args()


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


def cpu_baseline(n_nodes, seed, target_s):
    """Oracle (C restatement, OpenMP) on all nodes x a pod prefix, host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # checker only; never on the measured GPU path

    from minisched_amd import synth

    from minisched_amd.hostinfo import cpu_share

    share = cpu_share()  # the affinity mask, capped by the cgroup CPU quota
    threads = share["threads"]
    nr = synth.nodes(n_nodes, seed=seed)
    n_probe = 1024
    probe = synth.pods(n_probe, seed=seed)
    _oracle.schedule_nunn_omp(nr, probe[:64], seed=seed, threads=threads)  # thread pool warm-up
    t0 = time.perf_counter()
    _oracle.schedule_nunn_omp(nr, probe, seed=seed, threads=threads)
    dt = max(time.perf_counter() - t0, 1e-6)
    n_pods = int(min(1_000_000, max(n_probe, n_probe * target_s / dt)))
    pr = synth.pods(n_pods, seed=seed)
    t0 = time.perf_counter()
    _oracle.schedule_nunn_omp(nr, pr, seed=seed, threads=threads)
    dt = time.perf_counter() - t0
    faithful = cpu_faithful_1t(nr, n_nodes, seed, target_s / 4)
    return {
        "value": n_pods * n_nodes / dt,
        "unit": "pod×node evals/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle/ms_oracle.c msor_schedule_nunn_omp, {n_nodes} nodes x first {n_pods} pods "
        f"({dt:.1f} s, OpenMP {threads} threads); Go reference not buildable offline (GOMAXPROCS n/a)",
        "pods_per_s": n_pods / dt,
        "cpu_model": cpu_model(),
        "nproc": os.cpu_count(),
        "affinity_cpus": share["affinity"],
        "cgroup_quota_cpus": share["quota"],
        "threads_rule": "len(os.sched_getaffinity(0)), capped by the cgroup CPU quota (minisched_amd/hostinfo.py)",
        "faithful_1t": faithful,
    }


def cpu_faithful_1t(nr, n_nodes, seed, target_s):
    """SURVEY §8(d) cpu_faithful: one thread, the reference's per-pair work
    (last-character name parse per node and pod, per-pod feasible list, score
    list, then selectHost) — oracle/ms_oracle.c msor_schedule_nunn_names."""
    import _oracle  # checker only

    from minisched_amd import synth

    node_names = [f"node{i}" for i in range(n_nodes)]
    flags = np.ascontiguousarray(nr["unschedulable"], dtype=np.uint8)

    def run(n):
        pr = synth.pods(n, seed=seed)
        names = [f"pod{j}" for j in range(n)]
        t0 = time.perf_counter()
        _oracle.schedule_nunn_names(node_names, flags, names, pr["tolerates_unschedulable"], pr["ordinal"], seed=seed)
        return time.perf_counter() - t0

    dt = max(run(64), 1e-6)  # (the per-call ctypes name arrays are inside the clock, ~3 %)
    n = int(min(100_000, max(64, 64 * target_s / dt)))
    dt = run(n)
    return {"value": n * n_nodes / dt, "unit": "pod×node evals/s", "cores": 1, "kind": "port",
            "sample": f"msor_schedule_nunn_names, {n_nodes} node names x first {n} pods ({dt:.1f} s, 1 thread)",
            "pods_per_s": n / dt}


def timed(fn, stream, reps):
    """Mean device time of fn() on `stream` (HIP events around back-to-back launches)."""
    import torch

    fn()  # warm
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / reps


def timed_steady(fn, stream, block=10, tol=0.005, max_blocks=40):
    """The dominant kernel alone at steady clocks, measured BEFORE the warm-up steps.

    An idle MI355X ramps its clocks over the first ~10 ms of work: a kernel trace of
    the driver's shape (--steps 20 --warmup 5, profiles/r06a_timed_region.json) shows
    K1 launches shortening monotonically 272 -> 248 us over the first 36 launches, and
    a first step after 200 ms idle +113 us. That ramp, not a one-off in the loop, made
    device_ms_per_step exceed kernel_ms (timed after the region) by 3.4 % in BENCH_r05.
    So the kernel-alone measurement runs first, in blocks of `block` event-timed
    launches until the last three blocks agree within `tol` (at most `max_blocks`),
    which also brings the clocks up before the warm-up steps and the timed region.
    Returns (ms of the last block, every block's ms)."""
    hist = [timed(fn, stream, block) for _ in range(3)]
    while len(hist) < max_blocks and max(hist[-3:]) > (1.0 + tol) * min(hist[-3:]):
        hist.append(timed(fn, stream, block))
    return hist[-1], hist


def e2e_host(eng, pods_np, n_nodes, world=1, compact=False):
    """SURVEY §8(d) / BASELINE.md §2 pods/s: ms_schedule_batch on host arrays (H2D
    of the pods, the cycle, bind commit, D2H of the results), 1 warm-up then the
    median of 5; compact=True: ms_schedule_batch_compact (8 B per pod each way).
    With N > 1 the call is collective over the in-library communicator: every
    rank passes the same pods and receives every result."""
    import torch.distributed as dist

    from minisched_amd import _lib

    if compact:
        pods_np = _lib.compact_pods(pods_np)
        out = np.zeros(len(pods_np), dtype=_lib.RESULT_COMPACT)
        call = lambda: eng.schedule_compact(pods_np, _lib.MODE_BATCHED, out=out)  # noqa: E731
    else:
        out = np.zeros(len(pods_np), dtype=_lib.RESULT)
        call = lambda: eng.schedule(pods_np, _lib.MODE_BATCHED, out=out)  # noqa: E731
    call()
    ts, phases = [], []
    for _ in range(5):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
        # host phase times inside the call (ms_last_call_profile, us)
        phases.append({k: round(v, 1) if k != "chunks" else v for k, v in eng.last_call_profile().items()})
    ms = float(np.median(ts)) * 1e3
    P = len(pods_np)
    return {"ms_median": ms, "pods_per_s": P / (ms * 1e-3), "evals_per_s": P * n_nodes / (ms * 1e-3),
            "runs": [t * 1e3 for t in ts], "max_over_median": max(ts) / float(np.median(ts)),
            "phases_us": phases,
            "includes": ("ms_schedule_batch_compact: 8 B pods copied from the (pageable) host array into pinned "
                         "memory the kernel reads over PCIe (single shard; a staged H2D with N > 1)" if compact else
                         "ms_schedule_batch: H2D of 40 B pods (pageable host array)")
                        + ", filter+score+selectHost+decode"
                        + (", reduce-scatter + all-gather over the communicator" if world > 1 else "")
                        + ", bind commit, " + ("8 B results written by the kernel to pinned memory and copied into "
                                               "the host array" if compact else
                                               "D2H of 24 B results into the host array")}


def _cpu_info(threads):
    return {"cores": threads, "cpu_model": cpu_model(), "nproc": os.cpu_count()}


def _median_time(fn, reps=5, before=None, sync=None):
    """1 warm-up, then the median wall time of `reps` runs (before() untimed)."""
    if before:
        before()
    fn()
    if sync:
        sync()
    ts = []
    for _ in range(reps):
        if before:
            before()
        t0 = time.perf_counter()
        fn()
        if sync:
            sync()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def other_configs(args, dev, stream):
    """BASELINE.json's other configs on this GPU, each with a same-run CPU
    baseline: B 5k x 10k NU+NN exact sequential (CPU in full),
    D 50k x 1M NU+NN batched (CPU on a pod prefix), E 50k x 200k resource-aware
    exact sequential (CPU on an exact 2,000-pod prefix of the queue). Device
    figures: inputs resident in HBM, the engine's context stream, 1 warm-up then
    the median of 5 (B: of 21, a ~20 us call; B and E reset the node table before
    each run, untimed)."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # checker / CPU baseline only; never on the measured GPU path

    from minisched_amd import _lib, synth

    from minisched_amd.hostinfo import cpu_threads

    threads = cpu_threads()
    out = {}
    sync = torch.cuda.synchronize

    # ---- B: 5k nodes x 10k pods, NU+NN, exact sequential (assume-on-select binds)
    N, P = 5_000, 10_000
    nr, pr = synth.nodes(N, seed=args.seed), synth.pods(P, seed=args.seed)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, seed=args.seed, device=dev.index) as e:
        def reset():
            e.upsert(np.arange(N), nr)
            e.flush()
        # (a ~20 us call timed by host wall: 21 runs for a stable median)
        med, ts = _median_time(lambda: e.schedule_sequential_device(P, pods.data_ptr(), res.data_ptr()),
                               reps=21, before=reset, sync=sync)
        got = res.cpu().numpy().view(_lib.RESULT)
    t0 = time.perf_counter()
    o = _oracle.schedule(nr, pr, plugin_set=0, mode=1, seed=args.seed)
    cpu_seq = time.perf_counter() - t0
    names = [f"node{i}" for i in range(N)]
    t0 = time.perf_counter()
    _oracle.schedule_nunn_names(names, np.ascontiguousarray(nr["unschedulable"]), [f"pod{j}" for j in range(P)],
                                pr["tolerates_unschedulable"], pr["ordinal"], seed=args.seed)
    cpu_faithful = time.perf_counter() - t0
    t0 = time.perf_counter()
    _oracle.schedule_nunn_omp(nr, pr, seed=args.seed, threads=threads)
    cpu_omp = time.perf_counter() - t0
    out["B"] = {
        "workload": "B: 5000 nodes x 10000 pods, NU+NN, exact sequential (binds committed in queue order)",
        "ms": med * 1e3, "runs_ms": [t * 1e3 for t in ts], "evals_per_s": N * P / med, "pods_per_s": P / med,
        "parity_vs_oracle": bool(np.array_equal(got["node"], o["node"]) and np.array_equal(got["code"], o["code"])),
        "cpu_baseline": dict(value=N * P / cpu_faithful, unit="pod×node evals/s", kind="port",
                             sample=f"oracle msor_schedule_nunn_names (1 thread, per-pair name parse as "
                                    f"nodenumber.go:81-87), all {P} pods ({cpu_faithful:.2f} s)",
                             soa_1t=N * P / cpu_seq, omp=N * P / cpu_omp, omp_threads=threads,
                             **_cpu_info(1)),
    }

    # ---- C_names: config C with i.i.d. node-name digits (names unrelated
    # to the informer's Add order), ordinals from the digit-aligned allocator (encode.DigitOrdinals,
    # the shim's OrdinalAllocator): the layout a real cluster gives K1's fixed-slot form, beside
    # the synthetic cycling names of the headline (digit = ordinal % 10)
    from minisched_amd import encode

    N = P = 100_000
    base = synth.nodes(N, seed=args.seed)
    rng = np.random.default_rng(12345)
    base["name_digit"] = rng.integers(0, 10, N).astype(np.uint8)
    alloc = encode.DigitOrdinals(N + N // 10)
    ords = np.array([alloc.allocate(int(d)) for d in base["name_digit"]], dtype=np.uint32)
    pr = synth.pods(P, seed=args.seed)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=int(alloc.high), seed=args.seed, device=dev.index) as e:
        e.upsert(ords, base)
        e.flush()
        run = lambda: e.select_batch_device(P, pods.data_ptr(), res.data_ptr(), stream.cuda_stream)  # noqa: E731
        kms, _blocks = timed_steady(run, stream)
        got = res.cpu().numpy().view(_lib.RESULT)
    table = np.zeros(int(alloc.high), dtype=base.dtype)  # the oracle's records at the allocated ordinals
    table["allowed_pods"] = -1  # holes: never added, absent from the LIST
    table[ords] = base
    n_chk = 4096
    o = _oracle.schedule_nunn_omp(table, pr[:n_chk], seed=args.seed, threads=threads)
    out["C_names"] = {
        "workload": "C_names: config C (100000 nodes x 100000 pods, NU+NN, one fused launch) with i.i.d. node-name "
                    "digits, ordinals from the digit-aligned allocator in Add order",
        "ms": kms, "rows": int(alloc.high), "evals_per_s": N * P / (kms * 1e-3),
        "vs_cycling_names": None,
        "parity_vs_oracle_prefix": bool(all(np.array_equal(got[a][:n_chk].astype(np.int64), o[b].astype(np.int64))
                                            for a, b in (("node", "node"), ("code", "code"), ("score", "score"),
                                                         ("plugin_mask", "mask")))),
        "parity_pods": n_chk,
        "timing": "HIP events, blocks of 10 launches until three agree within 0.5 % (timed_steady)",
    }
    del pods, res

    # ---- D: 50k nodes x 1M pods, NU+NN, batched (stateless), one fused launch
    N, P = 50_000, 1_000_000
    nr, pr = synth.nodes(N, seed=args.seed), synth.pods(P, seed=args.seed)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, seed=args.seed, device=dev.index) as e:
        e.upsert(np.arange(N), nr)
        e.flush()
        med, ts = _median_time(lambda: e.select_batch_device(P, pods.data_ptr(), res.data_ptr()), sync=sync)
        got = res.cpu().numpy().view(_lib.RESULT)[:4096]
    n_omp = 20_000  # pod prefix for the CPU legs (prefix-extrapolated)
    t0 = time.perf_counter()
    o = _oracle.schedule_nunn_omp(nr, pr[:n_omp], seed=args.seed, threads=threads)
    cpu_omp = time.perf_counter() - t0
    n_f = 2_000
    names = [f"node{i}" for i in range(N)]
    t0 = time.perf_counter()
    _oracle.schedule_nunn_names(names, np.ascontiguousarray(nr["unschedulable"]), [f"pod{j}" for j in range(n_f)],
                                pr["tolerates_unschedulable"][:n_f], pr["ordinal"][:n_f], seed=args.seed)
    cpu_faithful = time.perf_counter() - t0
    out["D"] = {
        "workload": "D: 50000 nodes x 1000000 pods, NU+NN, batched (stateless), one fused launch",
        "ms": med * 1e3, "runs_ms": [t * 1e3 for t in ts], "evals_per_s": N * P / med, "pods_per_s": P / med,
        "parity_vs_oracle_prefix": bool(np.array_equal(got["node"], o["node"][:4096])),
        "cpu_baseline": dict(value=N * n_omp / cpu_omp, unit="pod×node evals/s", kind="port",
                             sample=f"oracle msor_schedule_nunn_omp ({threads} threads), first {n_omp} pods, "
                                    f"prefix-extrapolated ({cpu_omp:.2f} s)",
                             faithful_1t=N * n_f / cpu_faithful, faithful_sample=f"first {n_f} pods",
                             **_cpu_info(threads)),
    }
    del pods, res

    # ---- E: 50k nodes x 200k pods, NU+NRF+NN+LA, exact sequential (assume-on-select)
    N, P = 50_000, 200_000
    nr, pr = synth.nodes(N, seed=args.seed, resources=True), synth.pods(P, seed=args.seed, resources=True)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_NRF_NN_LA, seed=args.seed, device=dev.index) as e:
        def reset():
            e.upsert(np.arange(N), nr)
            e.flush()
        med, ts = _median_time(lambda: e.schedule_sequential_device(P, pods.data_ptr(), res.data_ptr()),
                               before=reset, sync=sync)
        got = res.cpu().numpy().view(_lib.RESULT)
        inf = e.info()
    n_pre = 2_000
    t0 = time.perf_counter()
    o = _oracle.schedule(nr, pr[:n_pre], plugin_set=1, mode=1, seed=args.seed)
    cpu_e = time.perf_counter() - t0
    n_batches = (P + 127) // 128
    line = {
        "workload": "E: 50000 nodes x 200000 pods, NU+NRF+NN+LA, exact sequential (assume-on-select), "
                    "speculative sweep + in-order validator, 128-pod batches",
        "ms": med * 1e3, "runs_ms": [t * 1e3 for t in ts], "evals_per_s": N * P / med, "pods_per_s": P / med,
        "us_per_batch": med * 1e6 / n_batches, "ns_per_pod": med * 1e9 / P,
        "parity_vs_oracle_prefix": bool(np.array_equal(got["node"][:n_pre], o["node"])
                                        and np.array_equal(got["code"][:n_pre], o["code"])),
        "fit_errors": int((got["code"] == _lib.CODE_UNSCHEDULABLE).sum()),
        "seq_counters_all_runs": dict(pods=inf.seq_pods, resweep_tiles=inf.seq_resweep_tiles,
                                      recomputes=inf.seq_recomputes, overflow=inf._pad),
        "cpu_baseline": dict(value=N * n_pre / cpu_e, unit="pod×node evals/s", kind="port",
                             sample=f"oracle msor_schedule (1 thread, exact sequential with binds), first "
                                    f"{n_pre} pods of the queue ({cpu_e:.2f} s)",
                             pods_per_s=n_pre / cpu_e, **_cpu_info(1)),
    }
    pj = None
    try:
        pj = json.load(open(args.profile_json_e))
    except Exception:
        pass
    # the step's two paths over a whole run (timeline build, tools/e_wg_timeline.py):
    # validator end V and merge-path end M from the step's start, and how often V is later
    step_split = None
    try:
        with open(os.path.join(ROOT, "profiles", "r06ag_e_wg_timeline_run.json")) as f:
            run = json.load(f)["run"]
        step_split = {k: run[k] for k in ("step_us_mean", "V_mean", "M_mean", "frac_validator_critical",
                                          "gap_us_mean")}
        step_split["profile"] = "profiles/r06ag_e_wg_timeline_run.json"
    except Exception:
        pass
    if pj and pj.get("nodes") == N and pj.get("pods") == P:
        step_s = pj["step_avg_ns_rocprof"] * 1e-9
        valu = pj["step_SQ_INSTS_VALU"]
        line["roofline"] = {
            "bound": "valu", "kernel": "k_seq_step",
            "achieved": valu / step_s, "peak": VALU_PEAK_NOMINAL, "unit": "wave-instr/s",
            "frac": valu / step_s / VALU_PEAK_NOMINAL,
            "frac_vs_guide_peak": valu / step_s / VALU_PEAK_GUIDE,
            "valu_insts_per_launch": valu, "kernel_ms_rocprof": step_s * 1e3,
            "step_split": step_split,
            "traffic": pj.get("step_hbm_bytes"),
            "fetch_bytes_per_step": pj.get("step_FETCH_SIZE_KB", 0) * 1024 * 2 or None,  # (gfx950 x2 read correction)
            "write_bytes_per_step": pj.get("step_WRITE_SIZE_KB", 0) * 1024 or None,
            "hbm": {"algorithmic_bytes_per_eval": BYTES_PER_EVAL["NU+NRF+NN+LA"],
                    "algorithmic_GBps": N * P * BYTES_PER_EVAL["NU+NRF+NN+LA"] / med / 1e9},
            "profile": os.path.relpath(args.profile_json_e, ROOT),
        }
    out["E"] = line
    del pods, res

    # ---- TT (not a BASELINE config): TaintToleration filter + the in-loop
    # reverse-normalised score (MS_PLUGINS_NU_TT_NN), 50k nodes x 100k pods, batched
    N, P = 50_000, 100_000
    nr, pr = synth.nodes(N, seed=args.seed, taints=True), synth.pods(P, seed=args.seed, taints=True)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_TT_NN, seed=args.seed, device=dev.index) as e:
        e.upsert(np.arange(N), nr)
        e.flush()
        med, ts = _median_time(lambda: e.select_batch_device(P, pods.data_ptr(), res.data_ptr()), sync=sync)
        got = res.cpu().numpy().view(_lib.RESULT)
    n_pre = 2_000
    t0 = time.perf_counter()
    o = _oracle.schedule_tt(nr, pr[:n_pre], literal=False, seed=args.seed)
    cpu_tt = time.perf_counter() - t0
    out["TT"] = {
        "workload": "TT (extension, not a BASELINE config): 50000 nodes x 100000 pods, NU+TaintToleration filters, "
                    "NN + TaintToleration score with the in-loop reverse DefaultNormalizeScore, batched",
        "ms": med * 1e3, "runs_ms": [t * 1e3 for t in ts], "evals_per_s": N * P / med, "pods_per_s": P / med,
        "parity_vs_oracle_prefix": bool(np.array_equal(got["node"][:n_pre], o["node"])
                                        and np.array_equal(got["code"][:n_pre], o["code"])),
        "cpu_baseline": dict(value=N * n_pre / cpu_tt, unit="pod×node evals/s", kind="port",
                             sample=f"oracle msor_schedule_tt closed form (1 thread), first {n_pre} pods "
                                    f"({cpu_tt:.2f} s)", pods_per_s=n_pre / cpu_tt, **_cpu_info(1)),
    }
    del pods, res

    # ---- NAM (not a BASELINE config): NodeAffinity with up to four preferred
    # terms per pod (raw scores to 400) through the in-loop DefaultNormalizeScore, 50k x 100k
    n_sets = 64
    nr = synth.nodes(N, seed=args.seed, labels=True)
    pr = synth.pods(P, seed=args.seed, term_sets=n_sets)
    ts = synth.nam_term_sets(n_sets, seed=args.seed)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_NN_NAM, seed=args.seed, device=dev.index) as e:
        e.nam_term_sets(ts)
        e.upsert(np.arange(N), nr)
        e.flush()
        med, ts_run = _median_time(lambda: e.select_batch_device(P, pods.data_ptr(), res.data_ptr()), sync=sync)
        got = res.cpu().numpy().view(_lib.RESULT)
    t0 = time.perf_counter()
    o = _oracle.schedule_nam(nr, pr[:n_pre], ts, literal=False, seed=args.seed)
    cpu_nam = time.perf_counter() - t0
    out["NAM"] = {
        "workload": "NAM (extension, not a BASELINE config): 50000 nodes x 100000 pods, NU filter, NN + NodeAffinity "
                    f"with up to 4 preferred terms per pod ({n_sets} term sets, raw scores to 400) and the in-loop "
                    "DefaultNormalizeScore, batched",
        "ms": med * 1e3, "runs_ms": [t * 1e3 for t in ts_run], "evals_per_s": N * P / med, "pods_per_s": P / med,
        "parity_vs_oracle_prefix": bool(np.array_equal(got["node"][:n_pre], o["node"])
                                        and np.array_equal(got["code"][:n_pre], o["code"])
                                        and np.array_equal(got["score"][:n_pre].astype(np.int64),
                                                           o["score"].astype(np.int64))),
        "cpu_baseline": dict(value=N * n_pre / cpu_nam, unit="pod×node evals/s", kind="port",
                             sample=f"oracle msor_schedule_nam closed form (1 thread), first {n_pre} pods "
                                    f"({cpu_nam:.2f} s)", pods_per_s=n_pre / cpu_nam, **_cpu_info(1)),
    }
    # ---- NAM_ext: the same shape with term sets in general form (ABI 7: In / NotIn / Exists /
    # DoesNotExist / Gt / Lt value-id sets, several requirements per term, synth.nam_term_sets_ext)
    nr = synth.nodes(N, seed=args.seed, labels=True)
    pr = synth.pods(P, seed=args.seed, term_sets=n_sets)
    tse = synth.nam_term_sets_ext(n_sets, seed=args.seed)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_NN_NAM, seed=args.seed, device=dev.index) as e:
        e.nam_term_sets_ext(tse)
        e.upsert(np.arange(N), nr)
        e.flush()
        med, ts_run = _median_time(lambda: e.select_batch_device(P, pods.data_ptr(), res.data_ptr()), sync=sync)
        got = res.cpu().numpy().view(_lib.RESULT)
    t0 = time.perf_counter()
    o = _oracle.schedule_nam_ext(nr, pr[:n_pre], tse, literal=False, seed=args.seed)
    cpu_name = time.perf_counter() - t0
    out["NAM_ext"] = {
        "workload": "NAM_ext (extension): NAM's shape with general preferred terms (In / NotIn / Exists / "
                    f"DoesNotExist / Gt / Lt, several requirements per term; {n_sets} term sets), batched",
        "ms": med * 1e3, "runs_ms": [t * 1e3 for t in ts_run], "evals_per_s": N * P / med, "pods_per_s": P / med,
        "parity_vs_oracle_prefix": bool(np.array_equal(got["node"][:n_pre], o["node"])
                                        and np.array_equal(got["code"][:n_pre], o["code"])
                                        and np.array_equal(got["score"][:n_pre].astype(np.int64),
                                                           o["score"].astype(np.int64))),
        "cpu_baseline": dict(value=N * n_pre / cpu_name, unit="pod×node evals/s", kind="port",
                             sample=f"oracle msor_schedule_nam_ext closed form (1 thread), first {n_pre} pods "
                                    f"({cpu_name:.2f} s)", pods_per_s=n_pre / cpu_name, **_cpu_info(1)),
    }
    return out


def slice_parity(n_nodes, seed, pods_np, a, b, res, threads, prefix=1024):
    """Checker, after the timed region: this rank's decoded pod slice [a, b) of
    the last timed batch against the oracle's OpenMP result over the WHOLE
    cluster (all n_nodes, every shard), on a prefix of the slice. Never on the
    measured path (the N > 1 line verifies itself)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # checker only

    from minisched_amd import synth

    k = int(min(prefix, b - a))
    if k <= 0:
        return {"ok": True, "n": 0}
    o = _oracle.schedule_nunn_omp(synth.nodes(n_nodes, seed=seed), pods_np[a:a + k], seed=seed, threads=threads)
    ok = all(np.array_equal(np.asarray(res[x][:k]).astype(np.int64), np.asarray(o[y]).astype(np.int64))
             for x, y in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")))
    return {"ok": bool(ok), "n": k}


RANK_FIELDS = ("rank", "comm_rank", "comm_world", "wall_s", "device_ms_per_step", "kernel_ms", "parity_ok",
               "parity_pods", "slice_first", "slice_end", "pods_scheduled")


def gather_rows(row, world, dev):
    """Every rank's RANK_FIELDS row on every rank (one all-gather, after the timed region)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [list(row)]
    t = torch.tensor(row, dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def load_profile(path, n_local, n_pods):
    try:
        pj = json.load(open(path))
    except Exception:
        return None
    if pj.get("kernel") != PP_KERNEL or pj.get("nodes") != n_local or pj.get("pods") != n_pods:
        return None
    return pj


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from minisched_amd import _lib, sharded, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # MINISCHED_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # cards round-robin); the driver's real runs use RCCL ("nccl"), one GPU per rank.
    backend = os.environ.get("MINISCHED_DIST_BACKEND", "nccl")
    local_dev = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    cfg = synth.CONFIGS[args.config]
    N, P = cfg["nodes"], cfg["pods"]
    if args.scaling == "weak":
        P = P * world  # the job's pod batch: the config's batch per GPU, same node count
    plugins = cfg["plugins"]
    split = args.split or ("pods" if args.config == "D" else "nodes")
    lo, hi = sharded.shard_bounds(N, rank, world) if split == "nodes" else (0, N)

    eng = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NN, node_base=lo, seed=args.seed,
                      device=local_dev)
    eng.upsert(np.arange(lo, hi, dtype=np.uint32), synth.nodes(hi - lo, seed=args.seed, start=lo))
    eng.flush()
    # N > 1 node split over RCCL: the in-library communicator (the Go-bindable path);
    # gloo rehearsals keep the Python combine
    use_lib = world > 1 and split == "nodes" and backend == "nccl"
    if use_lib:
        try:
            sharded.init_comm(eng)
        except _lib.MSError as ex:  # fail loudly: a timed line without the RCCL path would be meaningless
            print(f"bench.py rank {rank}/{world}: ms_comm_init failed ({_lib.ERRNAMES.get(ex.code, ex.code)}): {ex}",
                  file=sys.stderr, flush=True)
            raise SystemExit(3 if ex.code == _lib.MS_E_RCCL else 4)
        inf = eng.info()
        if (inf.comm_rank, inf.comm_world) != (rank, world):
            print(f"bench.py rank {rank}: the communicator reports rank {inf.comm_rank} of {inf.comm_world}, "
                  f"expected {rank} of {world}", file=sys.stderr, flush=True)
            raise SystemExit(3)
    present = sharded.present_total(eng) if split == "nodes" and not use_lib else None

    pods_np = synth.pods(P, seed=args.seed)
    pods = torch.from_numpy(pods_np.view(np.uint8).copy()).to(dev)
    # a real (non-null) stream: ms_* treat a NULL stream as the context's own
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    depth = int(os.environ.get("MINISCHED_PIPE_DEPTH", "4"))
    cyc = sharded.ShardedCycle(eng, N, P, pods, stream, split=split, depth=depth,
                               drain_group=int(os.environ.get("MINISCHED_PIPE_GROUP", str(depth))),
                               rank=rank, world=world, present_total=present)

    # the dominant kernel alone, on the step stream, at steady clocks (timed_steady:
    # measured before the warm-up steps): the fused cycle (N = 1 or pod split) or this
    # rank's sweep (node split)
    if cyc.library:
        kbuf = torch.empty(P, dtype=torch.int64, device=dev)
        kernel_fn = lambda: eng.sweep_device(P, pods.data_ptr(), kbuf.data_ptr(), 0, stream.cuda_stream)  # noqa: E731
        kernel_evals = float(P) * float(hi - lo)
    elif cyc._collective:
        kernel_fn = lambda: cyc.sweep(0)  # noqa: E731
        kernel_evals = float(P) * float(hi - lo)
    else:
        kernel_fn = cyc.step
        kernel_evals = float(cyc.b - cyc.a) * float(hi - lo)
    kernel_ms, kernel_blocks = timed_steady(kernel_fn, stream)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        cyc.step()
    cyc.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # device time of the timed region: one event pair on the step stream around all K steps
    ev_begin, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_begin.record(stream)
    for _ in range(args.steps):
        cyc.step()
    cyc.finish()  # node split: the last steps' combines + decodes
    ev_end.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_rank = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    step_dev_ms = ev_begin.elapsed_time(ev_end) / args.steps
    res = cyc.results.cpu().numpy().view(_lib.RESULT)[: cyc.b - cyc.a]
    ok = int((res["code"] == _lib.CODE_SUCCESS).sum())
    if world > 1:
        t = torch.tensor([ok], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        ok = int(t.item())

    # self-verification (after the timed region): the rank's communicator, its own
    # step times and the parity of its decoded slice; gathered to rank 0
    from minisched_amd.hostinfo import cpu_threads

    inf = eng.info()
    chk = slice_parity(N, args.seed, pods_np, cyc.a, cyc.b, res, max(1, cpu_threads() // max(1, world)))
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    rows = gather_rows([rank, inf.comm_rank, inf.comm_world if use_lib else -1, elapsed_rank, step_dev_ms, kernel_ms,
                        1.0 if chk["ok"] else 0.0, chk["n"], cyc.a, cyc.b,
                        int((res["code"] == _lib.CODE_SUCCESS).sum())], world, coll_dev)
    per_rank = [{k: (int(v) if k not in ("wall_s", "device_ms_per_step", "kernel_ms") else v)
                 for k, v in zip(RANK_FIELDS, r)} for r in rows]
    for r in per_rank:
        r["parity_ok"] = bool(r["parity_ok"])
        r["ms_per_step"] = r.pop("wall_s") * 1e3 / args.steps
    parity_all = all(r["parity_ok"] for r in per_rank)

    extras = {}
    if not args.no_extras:
        # SURVEY §8(d) pods/s: ms_schedule_batch on host arrays (collective with N > 1)
        for key, compact in (("e2e_compact", True), ("e2e", False)):
            try:
                extras[key] = e2e_host(eng, pods_np, N, world, compact=compact)
            except Exception as ex:  # (reported, never fatal to the headline line)
                extras[key] = {"error": repr(ex)[:300]}

    if rank == 0:
        ms_step = elapsed * 1e3 / args.steps
        value = float(P) * float(N) * args.steps / elapsed
        algo_bytes = kernel_evals * BYTES_PER_EVAL[plugins]
        kernel_s = kernel_ms * 1e-3
        # N > 1: this rank's shard sweep, counters of the same shard shape (tools/profile_shards.sh)
        prof_path = args.profile_json if world == 1 else f"{args.profile_shard_prefix}{hi - lo}.json"
        pj = load_profile(prof_path, hi - lo, P)
        valu = pj.get("SQ_INSTS_VALU") if pj else None
        traffic = pj.get("hbm_bytes_per_launch") if pj else None
        roofline = {
            "bound": "valu",
            "achieved": valu / kernel_s if valu else None,
            "peak": VALU_PEAK_NOMINAL,
            "unit": "wave-instr/s",
            "frac": (valu / kernel_s) / VALU_PEAK_NOMINAL if valu else None,
            "frac_of_measured_ceiling": (valu / kernel_s) / VALU_PEAK_MEASURED if valu else None,
            "peak_guide": VALU_PEAK_GUIDE,
            "frac_vs_guide_peak": (valu / kernel_s) / VALU_PEAK_GUIDE if valu else None,
            "peak_note": "peak = 4-cycle wave64 issue (the measured rate of every instruction K1 uses, "
                         + VALU_RATES_UBENCH + "); peak_guide = the guide's 2-cycle wave64 rate",
            "traffic": traffic,
            "kernel": PP_KERNEL,
            "kernel_ms": kernel_ms,
            # event-timed blocks of 10 launches before the warm-up, until three agree within 0.5 %
            # (timed_steady: the clock ramp of an idle GPU)
            "kernel_ms_blocks": [round(x, 5) for x in kernel_blocks],
            # the same kernel's average under rocprofv3 --kernel-trace (the committed summary; the profiler's
            # per-dispatch completion signals add a few %)
            "kernel_ms_rocprof": (pj.get("kernel_avg_ns_rocprof") or 0) * 1e-6 if pj else None,
            "valu_insts_per_launch": valu,
            "lane_valu_per_pair": valu * 64 / kernel_evals if valu else None,
            "profile": os.path.relpath(prof_path, ROOT) if pj else None,
            "hbm": {
                "algorithmic_bytes_per_launch": algo_bytes,
                "algorithmic_GBps": algo_bytes / kernel_s / 1e9,
                "dram_bytes_per_launch": traffic,
                "dram_GBps": traffic / kernel_s / 1e9 if traffic else None,
                "dram_frac": traffic / kernel_s / 1e9 / HBM_PEAK_GBS if traffic else None,
                "peak_GBps": HBM_PEAK_GBS,
                "note": "2 B/eval (SURVEY §8(d)) is re-read from registers: each workgroup loads the node bit "
                        "planes (0.75 B/node) once and evaluates ~200 pods against them, so the algorithmic "
                        "rate exceeds HBM peak by design and the kernel is VALU-issue bound",
            },
        }
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "pod×node evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic (splitmix64 seed {args.seed}, BASELINE.md §3)",
            "config": {
                "workload": f"{args.config}: {N} nodes x {P} pods ({P // world} per GPU, {args.scaling} scaling), "
                            f"{plugins}, batched, every pair evaluated, "
                            + (f"node-sharded over {world} GPU" if split == "nodes" else f"pods split over {world} GPU")
                            + (" (in-library RCCL communicator)" if cyc.library else ""),
                "nodes": N,
                "pods": P,
                "pods_per_gpu": P // world,
                "plugins": plugins,
                "parallelism": f"{'node' if split == 'nodes' else 'pod'}-shard{world}",
            },
            # pods/s = ms_schedule_batch wall time on host arrays (e2e); the
            # device-resident step rate separately
            "pods_per_s": (extras.get("e2e_compact") or {}).get("pods_per_s"),
            "device_pods_per_s": P * args.steps / elapsed,
            "device_ms_per_step": step_dev_ms,
            "pods_scheduled": ok,
            "roofline": roofline,
            "cpu_baseline": None,
            # each rank's communicator (RCCL rank / world as the
            # library reports them; -1 without the in-library communicator), its own
            # wall and device step times, its sweep kernel time, and the parity of its
            # decoded slice against the oracle over the whole cluster (a prefix of the
            # slice, checked after the timed region)
            "verify": {
                "backend": backend if world > 1 else None,
                "in_library_rccl": bool(cyc.library),
                "parity_ok_all_ranks": parity_all,
                "parity_check": "oracle msor_schedule_nunn_omp over all nodes, first <= 1024 pods of each rank's "
                                "decoded slice of the last timed batch (node, code, score, plugin mask)",
                "per_rank": per_rank,
            },
        }
        line.update(extras)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(N, args.seed, args.cpu_seconds)
        if world == 1 and not args.no_extras and not args.no_configs:
            try:
                line["configs"] = other_configs(args, dev, stream)
                cn = line["configs"].get("C_names")
                if cn:
                    cn["vs_cycling_names"] = cn["ms"] / kernel_ms  # (the headline kernel, same measurement)
            except Exception as ex:  # (reported, never fatal to the headline line)
                line["configs"] = {"error": repr(ex)[:300]}
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    if not parity_all:
        print(f"bench.py rank {rank}: decoded results differ from the oracle "
              f"({[r['rank'] for r in per_rank if not r['parity_ok']]})", file=sys.stderr, flush=True)
        raise SystemExit(5)


if __name__ == "__main__":
    main()
