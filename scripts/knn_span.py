"""KNN K4 span from a rocprofv3 kernel trace (--kernel-trace, csv): the launches of one rs_knn_sims
call overlap on two streams (the streamed download, sim.hip), so the per-kernel sums of
*_kernel_stats.csv over-count; the span is first knn_sims_mfma start -> last end.  Calls are split
at gaps > 50 ms.  Usage: python scripts/knn_span.py <run_kernel_trace.csv>"""
import csv
import sys


def spans(path):
    rows = [r for r in csv.DictReader(open(path))
            if "knn_sims_mfma" in r["Kernel_Name"] or "knn_scatter" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], []
    for r in rows:
        if cur and int(r["Start_Timestamp"]) - int(cur[-1]["End_Timestamp"]) > 50_000_000:
            groups.append(cur)
            cur = []
        cur.append(r)
    if cur:
        groups.append(cur)
    for g in groups:
        mf = [r for r in g if "mfma" in r["Kernel_Name"]]
        if not mf:
            continue
        t0 = min(int(r["Start_Timestamp"]) for r in g)
        m0 = min(int(r["Start_Timestamp"]) for r in mf)
        t1 = max(int(r["End_Timestamp"]) for r in g)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in mf)
        yield {"launches": len(mf), "streams": sorted({r["Stream_Id"] for r in mf}),
               "span_ms_with_scatter": (t1 - t0) / 1e6, "mfma_span_ms": (t1 - m0) / 1e6,
               "sum_of_mfma_durations_ms": busy / 1e6}


if __name__ == "__main__":
    for s in spans(sys.argv[1]):
        print(s)
