"""Config E against its golden fixture under the current environment (warm-up
batches / merge form); prints the mismatch count and the first differing pods."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-kube-scheduler_amd"))
from minisched_amd import _lib, synth  # noqa: E402

fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "config_e_full_seed1.npz"))
nr = synth.nodes(50_000, seed=1, resources=True)
pr = synth.pods(200_000, seed=1, resources=True)
for rep in range(int(os.environ.get("REPS", "2"))):
    with _lib.Engine(max_nodes=50_000, plugin_set=_lib.PLUGINS_NU_NRF_NN_LA, seed=1) as e:
        e.upsert(np.arange(50_000), nr)
        t0 = time.perf_counter()
        r = e.schedule(pr, _lib.MODE_SEQUENTIAL)
        dt = time.perf_counter() - t0
    bad = np.nonzero(r["node"].astype(np.int64) != fx["node"].astype(np.int64))[0]
    print(json.dumps({"warm": os.environ.get("MINISCHED_SEQ_WARM"), "merge": os.environ.get("MINISCHED_SEQ_MERGE"),
                      "rep": rep, "ms": round(dt * 1e3, 2), "n_bad": int(len(bad)),
                      "first": bad[:6].tolist()}), flush=True)
