"""Gap between kernel A's end (stream 1) and kernel B's start (stream 2) in a
rocprofv3 kernel trace of tools/ubench/xstream (python tools/ubench/xstream.py trace.csv)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# per iteration: C (s2), A (s1), B (s2), dispatched in that order
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"])) for r in rows]
by_stream = {}
for s, e, q in ks:
    by_stream.setdefault(q, []).append((s, e))
qs = sorted(by_stream, key=lambda q: len(by_stream[q]))
a_list = by_stream[qs[0]]  # stream 1: A only
cb = by_stream[qs[-1]]  # stream 2: C, B alternating
gaps_after_a, gaps_after_c = [], []
for i, (a_s, a_e) in enumerate(a_list[5:], start=5):
    c_s, c_e = cb[2 * i]
    b_s, b_e = cb[2 * i + 1]
    if c_e > a_e:
        gaps_after_c.append((b_s - c_e) / 1e3)
    else:
        gaps_after_a.append((b_s - a_e) / 1e3)
print(f"B start after A end (A last):  median {statistics.median(gaps_after_a):.2f} us  n={len(gaps_after_a)}")
print(f"B start after C end (C last):  median {statistics.median(gaps_after_c):.2f} us  n={len(gaps_after_c)}")
