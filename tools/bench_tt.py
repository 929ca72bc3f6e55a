"""The TT extension config alone (bench.py's `configs.TT`: 50k nodes x 100k
pods, MS_PLUGINS_NU_TT_NN, batched, device entry point): median of --reps timed
cycles and the oracle's closed form on a 2,000-pod prefix (checker). For A/Bs:
MINISCHED_TT=v1 selects the per-pair summary sweep."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from minisched_amd import _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--nodes", type=int, default=50_000)
ap.add_argument("--pods", type=int, default=100_000)
ap.add_argument("--seed", type=int, default=1)
args = ap.parse_args()
N, P = args.nodes, args.pods
dev = torch.device("cuda:0")
nr, pr = synth.nodes(N, seed=args.seed, taints=True), synth.pods(P, seed=args.seed, taints=True)
pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
ts = []
with _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_TT_NN, seed=args.seed, device=0) as e:
    e.upsert(np.arange(N), nr)
    e.flush()
    for i in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.select_batch_device(P, pods.data_ptr(), res.data_ptr())
        torch.cuda.synchronize()
        if i:
            ts.append(time.perf_counter() - t0)
    got = res.cpu().numpy().view(_lib.RESULT)
import _oracle  # noqa: E402  (checker)

o = _oracle.schedule_tt(nr, pr[:2000], literal=False, seed=args.seed)
ok = all(np.array_equal(got[k][:2000].astype(np.int64), o[ko].astype(np.int64))
         for k, ko in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")))
print(json.dumps({"tt": os.environ.get("MINISCHED_TT", "v2"), "median_ms": float(np.median(ts)) * 1e3,
                  "runs_ms": [t * 1e3 for t in ts], "evals_per_s": N * P / float(np.median(ts)), "parity_prefix": ok}))
