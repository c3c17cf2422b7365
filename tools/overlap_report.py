"""Overlap of collective kernels with compute kernels in a rocprofv3 kernel trace.

    python tools/overlap_report.py <..._kernel_trace.csv> [--compute u8_wgrad] [--comm nccl]

For every kernel whose name contains --comm (case-insensitive: RCCL's ncclDevKernel_* / rccl*), prints the
compute kernels (names containing --compute) whose [start, end) intersects it and the overlapped time."""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--compute", default="u8_wgrad")
    ap.add_argument("--comm", default="nccl")
    ap.add_argument("--last", type=int, default=6, help="report the last N collectives")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?"),
                         r.get("Stream_Id", "?")))
    rows.sort()
    comm = [r for r in rows if re.search(a.comm, r[2], re.I)]
    comp = [r for r in rows if a.compute in r[2]]
    print(f"{len(comm)} collective kernels, {len(comp)} compute kernels matching {a.compute!r}")
    tot_ov = 0
    for c in comm[-a.last:]:
        s, e = c[0], c[1]
        ov = []
        for k in comp:
            lo, hi = max(s, k[0]), min(e, k[1])
            if hi > lo:
                ov.append((k, hi - lo))
        tot_ov += sum(o for _, o in ov)
        print(f"collective {c[2][:60]} queue {c[3]} stream {c[4]}: {(e - s) / 1e3:.1f} us")
        for k, o in ov:
            print(f"   overlaps {k[2][:70]} (queue {k[3]}) for {o / 1e3:.1f} us")
    print(f"total overlapped collective time (last {min(a.last, len(comm))}): {tot_ov / 1e3:.1f} us")


if __name__ == "__main__":
    main()
