#!/usr/bin/env python3
"""K1 pp at config C on node-naming layouts (skewed digits).

  cycling : node{i} at ordinal i (digit = i % 10, the synthetic default)
  iid     : digits i.i.d. uniform 0..9 (names unrelated to ordinals)
  perm    : ordinal i holds node{perm[i]} (informer Add order != name order)
  iid_allocated : the iid names, ordinals from the digit-aligned allocator
            (encode.DigitOrdinals, the host mirror's OrdinalAllocator) in Add
            order; the table spans the allocator's high-water mark (holes absent)
  skew_allocated / skew_dense : 70 % of the names end in 0, allocator ordinals
            (bounded spread) / ordinals in Add order (PROBE_LAYOUTS=a,b selects)

Each: mean device time of the fused single-launch cycle (ms_select_batch_device)
over K launches, the fraction of 30-row groups whose "over" plane is set (the
bit-scan path), and parity of every pod against the OpenMP oracle.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def layouts(n, seed):
    from minisched_amd import synth

    base = synth.nodes(n, seed=seed)
    rng = np.random.default_rng(12345)
    iid = base.copy()
    iid["name_digit"] = rng.integers(0, 10, n).astype(np.uint8)
    perm = base.copy()
    perm["name_digit"] = (rng.permutation(n) % 10).astype(np.uint8)
    from minisched_amd import encode

    alloc = encode.DigitOrdinals(n + n // 10)
    ords = np.array([alloc.allocate(int(d)) for d in iid["name_digit"]])
    allocated = np.zeros(alloc.high, dtype=base.dtype)
    allocated["allowed_pods"] = -1  # never added: absent from the LIST
    allocated[ords] = iid
    # skewed names (70 % end in 0): the allocator keeps digit-aligned ordinals only
    # within its bounded spread of the dense frontier, else the lowest free one
    skew = base.copy()
    skew["name_digit"] = np.where(rng.random(n) < 0.7, 0, rng.integers(0, 10, n)).astype(np.uint8)
    alloc2 = encode.DigitOrdinals(2 * n)
    ords2 = np.array([alloc2.allocate(int(d)) for d in skew["name_digit"]])
    skew_alloc = np.zeros(alloc2.high, dtype=base.dtype)
    skew_alloc["allowed_pods"] = -1
    skew_alloc[ords2] = skew
    out = {"cycling": base, "iid": iid, "perm": perm, "iid_allocated": allocated, "skew_allocated": skew_alloc,
           "skew_dense": skew}
    only = os.environ.get("PROBE_LAYOUTS")
    return {k: v for k, v in out.items() if not only or k in only.split(",")}


def misaligned_frac(nr):
    """Groups the fixed-slot form cannot take: a present digit-named row whose digit
    is not its ordinal mod 10."""
    ok = (nr["allowed_pods"] < 0) | (nr["name_digit"] > 9) | (nr["name_digit"] == np.arange(len(nr)) % 10)
    g = len(ok) // 30
    return float((~ok[: g * 30].reshape(g, 30).all(1)).mean())


def over_frac(nr):
    d = np.where(nr["allowed_pods"] >= 0, nr["name_digit"].astype(np.int64), 99)
    g = len(d) // 30
    d = d[: g * 30].reshape(g, 30)
    cnt = np.stack([(d == v).sum(1) for v in range(10)], 1)
    return float((cnt.max(1) > 3).mean())


def main():
    import torch

    import _oracle  # checker only
    from minisched_amd import _lib, synth

    N, P, K = 100_000, 100_000, int(os.environ.get("PROBE_REPS", 20))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pr = synth.pods(P, seed=1)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    out = {}
    for name, nr in layouts(N, 1).items():
        rows = len(nr)
        listed = np.nonzero(nr["allowed_pods"] >= 0)[0]
        with _lib.Engine(max_nodes=rows, seed=1) as e:
            e.upsert(listed, nr[listed])
            e.flush()
            run = lambda: e.select_batch_device(P, pods.data_ptr(), res.data_ptr(), s.cuda_stream)
            run()
            s.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(K):
                run()
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / K
            got = res.cpu().numpy().view(_lib.RESULT)
        t0 = time.perf_counter()
        o = _oracle.schedule_nunn_omp(nr, pr, seed=1, threads=16)
        ok = all(np.array_equal(got[a].astype(np.int64), o[b].astype(np.int64))
                 for a, b in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")))
        out[name] = {"ms": ms, "rows": rows, "evals_per_s": N * P / (ms * 1e-3), "over_group_frac": over_frac(nr), "misaligned_group_frac": misaligned_frac(nr),
                     "parity": ok, "oracle_s": time.perf_counter() - t0}
        print(name, json.dumps(out[name]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
