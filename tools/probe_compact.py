#!/usr/bin/env python3
"""ms_schedule_batch_compact at config C (100k nodes x 100k pods, host arrays):
median wall time of 21 calls and a digest of the results (MINISCHED_COMPACT_ZC
selects the zero-copy or the staged form; run one process per form)."""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    from minisched_amd import _lib, synth

    N = P = 100_000
    pods = _lib.compact_pods(synth.pods(P, seed=1))
    out = np.zeros(P, dtype=_lib.RESULT_COMPACT)
    with _lib.Engine(max_nodes=N, seed=1) as e:
        e.upsert(np.arange(N), synth.nodes(N, seed=1))
        e.flush()
        e.schedule_compact(pods, _lib.MODE_BATCHED, out=out)
        digest = hashlib.sha256(out.tobytes()).hexdigest()[:16]
        ts = []
        for _ in range(21):
            t0 = time.perf_counter()
            e.schedule_compact(pods, _lib.MODE_BATCHED, out=out)
            ts.append(time.perf_counter() - t0)
    print(json.dumps({"zc": os.environ.get("MINISCHED_COMPACT_ZC", "1"), "ms_median": round(float(np.median(ts)) * 1e3, 4),
                      "ms_min": round(min(ts) * 1e3, 4), "digest_first_call": digest}), flush=True)


if __name__ == "__main__":
    main()
