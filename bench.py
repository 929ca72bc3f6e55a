#!/usr/bin/env python3
"""Headline benchmark: minisched's scheduling cycle on MI355X.

Metric (BASELINE.json): pod x node filter+score evals/sec (and pods scheduled/sec)
at 100k nodes on 1/2/4/8 GPUs -> workload = config C: 100,000 nodes x
100,000 pods, NodeUnschedulable + NodeNumber, node-sharded across ranks with
one RCCL MAX all-reduce of the packed keys per step.

One step = the whole batch through the hot path with inputs resident in HBM:
  ms_sweep_device (fused filter->score->argmax over this rank's node shard)
  -> all_reduce(keys, MAX) over RCCL (N > 1)
  -> ms_decode_device (packed key -> node / code / score / FitError mask).
For N > 1 step k's all-reduce overlaps step k+1's sweep and step k's decode
follows it (two key buffers); the last step is drained before the clock stops.
value = P * N_total / step time (max over ranks), i.e. whole-job evals/s.

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 the driver
uses torch.distributed.run with one rank per GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))

METRIC = "pod×node filter+score evals/sec and pods scheduled/sec at 100k nodes, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_EVAL = {"NU+NN": 2, "NU+NRF+NN+LA": 58}
# rocprof kernel-name keys; the default (no MINISCHED_K1) is the production choice,
# k_sweep_nunn_v8 at 100k rows per GPU and k_sweep_nunn_v7 on small shards
K1_KERNELS = {"v0": "k_sweep_nunn<", "v7": "k_sweep_nunn_v7", "v8": "k_sweep_nunn_v8", None: "k_sweep_nunn_v"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C", choices=["B", "C", "D"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_C.json"))
    return ap.parse_args()


def cpu_baseline(n_nodes, seed, target_s):
    """Oracle (C restatement, OpenMP) on all nodes x a pod prefix, host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # checker only; never on the measured GPU path

    from minisched_amd import synth

    threads = min(16, os.cpu_count() or 1)  # the box's CPU share is 16
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
    if backend == "nccl":
        local_dev = local
    else:
        local_dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    cfg = synth.CONFIGS[args.config]
    N, P = cfg["nodes"], cfg["pods"]
    plugins = cfg["plugins"]
    lo, hi = sharded.shard_bounds(N, rank, world)  # this rank's node shard

    eng = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NN, node_base=lo, seed=args.seed,
                      device=local_dev)
    eng.upsert(np.arange(lo, hi, dtype=np.uint32), synth.nodes(hi - lo, seed=args.seed, start=lo))
    eng.flush()

    pods_np = synth.pods(P, seed=args.seed)
    pods = torch.from_numpy(pods_np.view(np.uint8).copy()).to(dev)
    # a real (non-null) stream: ms_* treat a NULL stream as the context's own
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    # N > 1: each step's RCCL all-reduce overlaps the following steps' sweeps
    # (sharded.CrossStepPipeline, depth 4: four all-reduces in flight, five key
    # buffers); every fourth step waits once, for the newest all-reduce, and
    # decodes four batches in one launch (ms_decode_device_jobs). A cross-queue
    # wait idles the sweep stream ~10 us however early its event completed
    # (profiles/r01t_pipeline_group_ab.jsonl, r01v_pipeline_group_decode_jobs_ab.jsonl).
    # The last steps' combines + decodes are drained inside the timed region.
    # MINISCHED_PIPE_DEPTH / MINISCHED_PIPE_GROUP / MINISCHED_DECODE_STREAM=1 select
    # the other measured forms; MINISCHED_BENCH_PIPE=0 falls back to in-step pod
    # chunks (MINISCHED_BENCH_CHUNKS) whose reductions overlap the next chunk's sweep.
    # N = 1 (MINISCHED_BENCH_PIPE1=1): the same pipeline with no collective, so
    # decodes launch in groups too
    pipe1 = world == 1 and os.environ.get("MINISCHED_BENCH_PIPE1", "0") == "1"
    pipe = (world > 1 or pipe1) and os.environ.get("MINISCHED_BENCH_PIPE", "1") != "0"
    chunks = int(os.environ.get("MINISCHED_BENCH_CHUNKS", "4" if world > 1 else "1"))
    cyc = sharded.ShardedCycle(eng, N, P, pods, stream, want_flags=False, chunks=chunks, pipeline=pipe,
                               decode_stream=os.environ.get("MINISCHED_DECODE_STREAM", "0") == "1",
                               depth=int(os.environ.get("MINISCHED_PIPE_DEPTH", "4")),
                               drain_group=int(os.environ.get("MINISCHED_PIPE_GROUP", "4")),
                               collective=world > 1)

    # Device time of the timed region: ONE event pair on the sweep stream around
    # all K steps. Per-step event records sit inside the timed region and cost
    # ~4 % of a step (profiles/r01z_n1_bench_forms_ab.jsonl);
    # MINISCHED_BENCH_STEP_EVENTS=1 brings them back for per-step spreads.
    per_step_events = os.environ.get("MINISCHED_BENCH_STEP_EVENTS", "0") == "1"
    sweep_events = []

    def step(timed):
        if timed and per_step_events:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            cyc.step(world)
            b.record(stream)
            sweep_events.append((a, b))
        else:
            cyc.step(world)

    for _ in range(args.warmup):
        step(False)
    cyc.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev_begin, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_begin.record(stream)
    for _ in range(args.steps):
        step(True)
    cyc.finish()  # pipelined: the last steps' combines + decodes
    ev_end.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if sweep_events:
        step_dev_ms = float(np.mean([a.elapsed_time(b) for a, b in sweep_events]))
    else:
        step_dev_ms = ev_begin.elapsed_time(ev_end) / args.steps
    # kernel-only timing on the sweep's stream: separate timed launches after the run
    kev = []
    for _ in range(max(3, min(args.steps, 10))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        cyc.sweep(0, P)
        b.record(stream)
        kev.append((a, b))
    torch.cuda.synchronize()
    sweep_ms = float(np.mean([a.elapsed_time(b) for a, b in kev]))
    res = cyc.results.cpu().numpy().view(_lib.RESULT)
    ok = int((res["code"] == _lib.CODE_SUCCESS).sum())

    if rank == 0:
        ms_step = elapsed * 1e3 / args.steps
        evals = float(P) * float(N)
        value = evals * args.steps / elapsed
        local_evals = float(P) * float(hi - lo)
        achieved = local_evals * BYTES_PER_EVAL[plugins] / (sweep_ms * 1e-3) / 1e9
        traffic, limiter, tj_kernel = None, None, None
        if os.path.exists(args.traffic_json) and world == 1:
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("kernel") == K1_KERNELS.get(os.environ.get("MINISCHED_K1")):
                    traffic = tj.get("hbm_bytes_per_launch")
                    tj_kernel = tj.get("kernel_name")  # the instance rocprof saw
                    # the sweep keeps node columns in registers, so issue, not HBM, binds it
                    limiter = {"kind": "VALU issue", "valu_busy_frac": tj.get("valu_busy_frac"),
                               "valu_insts_per_launch": tj.get("valu_insts_per_launch"),
                               "source": os.path.relpath(args.traffic_json, ROOT)}
            except Exception:
                traffic, limiter = None, None
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "pod×node evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": f"synthetic (splitmix64 seed {args.seed}, BASELINE.md §3)",
            "config": {
                "workload": f"{args.config}: {N} nodes x {P} pods, {plugins}, batched, node-sharded over {world} GPU",
                "nodes": N,
                "pods": P,
                "plugins": plugins,
                "parallelism": f"node-shard{world}",
            },
            "pods_per_s": P * args.steps / elapsed,
            "device_ms_per_step": step_dev_ms,
            "pod_chunks": len(cyc.chunks),
            "cross_step_pipeline": pipe,
            "pods_scheduled": ok,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": tj_kernel or K1_KERNELS.get(os.environ.get("MINISCHED_K1"), "k_sweep_nunn_v"),
                "kernel_ms": sweep_ms,
                "algorithmic_bytes_per_launch": local_evals * BYTES_PER_EVAL[plugins],
                "limiter": limiter,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(N, args.seed, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
