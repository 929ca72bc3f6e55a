#!/usr/bin/env python3
"""NodeAffinity extension timing (the NU+NN+NodeAffinity set): 50k
nodes x 100k pods, MS_PLUGINS_NU_NN_NA, one batched select per rep, and a parity
check of the first 1,000 pods against the oracle. MINISCHED_LIB selects a build."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import _oracle  # checker only
    from minisched_amd import _lib, synth

    N, P, K = 50_000, 100_000, 10
    dev = torch.device("cuda:0")
    nr, pr = synth.nodes(N, seed=1, zones=True), synth.pods(P, seed=1, zones=True)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    with _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_NN_NA, seed=1) as e:
        e.upsert(np.arange(N), nr)
        e.flush()
        e.select_batch_device(P, pods.data_ptr(), res.data_ptr())
        torch.cuda.synchronize()
        t0 = time.perf_counter()  # (the library runs on its own stream: device-wide sync)
        for _ in range(K):
            e.select_batch_device(P, pods.data_ptr(), res.data_ptr())
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        got = res.cpu().numpy().view(_lib.RESULT)
    o = _oracle.schedule_na(nr, pr[:1000], seed=1, literal=False)
    ok = bool(np.array_equal(got["node"][:1000], o["node"]) and np.array_equal(got["code"][:1000], o["code"]))
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "ms": ms, "parity_1000": ok}))


if __name__ == "__main__":
    main()
