"""Timeline summary of a rocprofv3 kernel (+ memory copy) trace of the bench
line: copy durations and rates, GPU-busy union, K3 concurrency, idle gaps.
Usage: python3 tools/tl_analyze.py <dir with run_kernel_trace.csv>"""
import csv, os, sys

d = sys.argv[1]
K = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in K]
k3 = sorted(e for e in ev if e[2].startswith("void k_encode"))
# steady state: from the 3rd K3 start to the last K3 end
t0, t1 = k3[min(2, len(k3) - 1)][0], k3[-1][1]
win = t1 - t0
print("window %.1f ms, %d K3 launches in it" % (win / 1e6, sum(1 for e in k3 if e[0] >= t0)))
def union(iv):
    iv = sorted((max(a, t0), min(b, t1)) for a, b, *_ in iv if b > t0 and a < t1)
    tot, cs, ce = 0, None, None
    for a, b in iv:
        if cs is None or a > ce:
            if cs is not None: tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if cs is not None: tot += ce - cs
    return tot
print("any kernel busy %.1f%%, K3 busy %.1f%%" % (100 * union(ev) / win, 100 * union(k3) / win))
# K3 concurrency
pts = sorted([(a, 1) for a, b, _ in k3] + [(b, -1) for a, b, _ in k3])
lvl, last, hist = 0, t0, {}
for t, dlt in pts:
    tt = min(max(t, t0), t1)
    hist[lvl] = hist.get(lvl, 0) + tt - last
    last, lvl = tt, lvl + dlt
print("K3 concurrency:", {k: "%.1f%%" % (100 * v / win) for k, v in sorted(hist.items())})
print("K3 durations ms:", [round((b - a) / 1e6, 1) for a, b, _ in k3])
mc = os.path.join(d, "run_memory_copy_trace.csv")
if os.path.exists(mc):
    M = list(csv.DictReader(open(mc)))
    if M:
        print("copy columns:", list(M[0].keys()))
    for r in M:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = int(r.get("Bytes", r.get("Size", 0)) or 0)
        if n > 50 << 20:
            print("  copy %-28s %7.1f MB %7.2f ms %6.1f GB/s  at %+.1f ms" % (
                r.get("Direction", r.get("Operation", "")), n / 1e6, (b - a) / 1e6,
                n / max(1, b - a), (a - t0) / 1e6))
