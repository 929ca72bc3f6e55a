#!/usr/bin/env python3
"""Interleaved A/B of NU+NN cycle forms in ONE process (perf deltas only from
interleaved rounds on one device).

AB_VARIANTS = "name:K=V,K=V;name2:K=V" — each variant sets those env vars
(read by the library at each launch) on top of the base environment.
AB_MODE = select (ms_select_batch_device: the fused single-shard cycle, default)
        | sweep  (ms_sweep_device: this shard's keys only)
        | sweepdec (ms_sweep_device + ms_decode_device: the unfused cycle);
a variant may set MODE=... itself (results of different modes are not compared).
Prints per-variant kernel ms (HIP events on the launch stream), median and
min over rounds, and whether all variants produced identical bytes."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def parse_variants(spec):
    out = []
    for item in spec.split(";"):
        item = item.strip()
        if not item:
            continue
        name, _, kv = item.partition(":")
        env = {}
        for pair in filter(None, kv.split(",")):
            k, _, v = pair.partition("=")
            env[k.strip()] = v.strip()
        out.append((name, env))
    return out


def main():
    import torch

    from minisched_amd import _lib, synth

    N = int(os.environ.get("AB_NODES", 100_000))
    P = int(os.environ.get("AB_PODS", 100_000))
    base_ord = int(os.environ.get("AB_NODE_BASE", 0))
    rounds = int(os.environ.get("AB_ROUNDS", 8))
    mode = os.environ.get("AB_MODE", "select")
    variants = parse_variants(os.environ.get("AB_VARIANTS", "pp:MINISCHED_K1=pp"))
    touched = {k for _, env in variants for k in env}
    base_env = {k: os.environ.get(k) for k in touched}
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    eng = _lib.Engine(max_nodes=N, seed=1, node_base=base_ord)
    eng.upsert(np.arange(base_ord, base_ord + N), synth.nodes(N, seed=1, start=base_ord))
    eng.flush()
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    outs = {n: torch.empty(P * 24, dtype=torch.uint8, device=dev) for n, _ in variants}
    keys = torch.empty(P, dtype=torch.int64, device=dev)
    times = {n: [] for n, _ in variants}
    for r in range(rounds + 1):
        for name, env in variants:
            vmode = env.get("MODE", mode)
            for k in touched:
                if k == "MODE":
                    continue
                if k in env:
                    os.environ[k] = env[k]
                elif base_env[k] is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = base_env[k]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            if vmode == "select":
                eng.select_batch_device(P, pods.data_ptr(), outs[name].data_ptr(), s.cuda_stream)
            elif vmode == "sweepdec":
                eng.sweep_device(P, pods.data_ptr(), keys.data_ptr(), 0, s.cuda_stream)
                eng.decode_device(P, pods.data_ptr(), keys.data_ptr(), 0, N, outs[name].data_ptr(), s.cuda_stream)
            else:
                eng.sweep_device(P, pods.data_ptr(), outs[name].data_ptr(), 0, s.cuda_stream)
            b.record(s)
            b.synchronize()
            if r:
                times[name].append(a.elapsed_time(b))
    names = [n for n, _ in variants]
    mode_of = {n: {"sweepdec": "select"}.get(env.get("MODE", mode), env.get("MODE", mode)) for n, env in variants}
    same = all(torch.equal(outs[names[0]], outs[n]) for n in names[1:] if mode_of[n] == mode_of[names[0]])
    out = {n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "evals_per_s": N * P / (np.median(t) * 1e-3)} for n, t in times.items()}
    out["identical"] = bool(same)
    out["nodes"], out["pods"], out["mode"] = N, P, mode
    print(json.dumps(out))


if __name__ == "__main__":
    main()
