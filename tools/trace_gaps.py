"""Device idle time in a rocprofv3 kernel trace: busy (union of kernel intervals, all queues) vs wall time over the
last N steps, and the largest idle gaps with the kernels on either side.

    python tools/trace_gaps.py <..._kernel_trace.csv> --marker sgd_mixed --steps 5 [--top 15]

A step ends at each kernel whose name contains --marker (the optimizer launch is the last kernel of a training
step); the window is the last --steps steps (from the end of the marker kernel --steps + 1 back)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sgd_mixed")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    ends = [e for s, e, n in rows if a.marker in n]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} marker kernels ({a.marker!r})")
    t0, t1 = ends[-a.steps - 1], ends[-1]
    win = [(max(s, t0), min(e, t1), n) for s, e, n in rows if e > t0 and s < t1]
    busy, gaps, cur_end, prev = 0, [], t0, "(step start)"
    for s, e, n in win:
        if s > cur_end:
            gaps.append((s - cur_end, prev, n))
        if e > cur_end:
            busy += e - max(s, cur_end)
            cur_end, prev = e, n
    wall = t1 - t0
    print(f"{a.steps} steps: wall {wall / 1e6 / a.steps:.3f} ms/step, busy {busy / 1e6 / a.steps:.3f} ms/step, "
          f"idle {(wall - busy) / 1e6 / a.steps:.3f} ms/step ({100 * (wall - busy) / wall:.1f} %), "
          f"{len(gaps) / a.steps:.1f} gaps/step")
    gaps.sort(reverse=True)
    for g, p, n in gaps[:a.top]:
        print(f"  {g / 1e3:8.1f} us  after {p[:70]}\n              before {n[:70]}")


if __name__ == "__main__":
    main()
