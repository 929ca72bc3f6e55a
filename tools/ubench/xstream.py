"""Gap between kernel B's start and the end of the kernels it waits for, in a
rocprofv3 kernel trace of tools/ubench/xstream (python tools/ubench/xstream.py trace.csv).
Per iteration the dispatches are C (s2), A (s1), B (s2, after A via the hand-off);
kernels are matched by dispatch order (the trace's stream ids are not reliable)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
gaps_after_a, gaps_after_c = [], []
for i in range(5, len(ks) // 3):
    (c_s, c_e), (a_s, a_e), (b_s, b_e) = ks[3 * i], ks[3 * i + 1], ks[3 * i + 2]
    if c_e > a_e:
        gaps_after_c.append((b_s - c_e) / 1e3)
    else:
        gaps_after_a.append((b_s - a_e) / 1e3)
for name, g in (("A last (waiting on the hand-off)", gaps_after_a), ("C last (hand-off already signalled)", gaps_after_c)):
    if g:
        print(f"B start - end of {name}: median {statistics.median(g):.2f} us  n={len(g)}")
