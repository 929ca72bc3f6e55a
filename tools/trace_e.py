"""Timeline summary of a config E kernel trace: per-kernel medians and the gaps
between consecutive validator launches (python tools/trace_e.py <trace.csv>)."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
for nm in ("k_validate_seq", "k_sweep_full_topk", "k_topk_merge"):
    d = [e - s for s, e, n, q in ks if nm in n]
    if d:
        print(f"{nm:20s} n={len(d):5d} median={statistics.median(d)/1e3:7.1f} us total={sum(d)/1e6:7.2f} ms")
val = [(s, e) for s, e, n, q in ks if "k_validate_seq" in n]
gaps = [val[i + 1][0] - val[i][1] for i in range(len(val) - 1)]
gaps = [g for g in gaps if g < 1e6]
print(f"validator-to-validator gap: median={statistics.median(gaps)/1e3:.1f} us, mean={statistics.mean(gaps)/1e3:.1f} us")
mid = len(ks) // 2
t0 = ks[mid][0]
for s, e, n, q in ks[mid:mid + 12]:
    print(f"{(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} {n.split('(')[0][-24:]:24s} stream {q}")
