"""Summaries of rocprofv3 output for profiles/ (kernel stats -> per-step table; PMC -> per-kernel
averages with derived utilisations).

    python tools/summarize_profile.py stats <kernel_stats.csv> <steps>
    python tools/summarize_profile.py pmc <counter_collection.csv> [more.csv ...]
    python tools/summarize_profile.py trace <kernel_trace.csv> <steps>   (rocpd2csv output of a .db run)
    python tools/summarize_profile.py db <run_results.db> <steps>        (rocprofv3's default rocpd output)
"""
import collections
import csv
import sys


def stats(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"kernel time per step: {tot / 1e6 / steps:.3f} ms over {steps} steps (incl. warm-up/setup kernels)")
    print(f"{'ms/step':>8} {'calls/step':>10} {'avg us':>9} {'%':>6}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e6 / steps:8.3f} {int(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:9.1f} "
              f"{100 * t / tot:6.2f}  {r['Name'][:120]}")


def trace(path, steps):
    """Per-kernel stats from a kernel-trace CSV (rocprofv3's default .db output, exported with
    rocpd2csv) in the same layout as `stats`."""
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values())
    print(f"kernel time per step: {tot / 1e6 / steps:.3f} ms over {steps} steps (incl. warm-up/setup kernels)")
    print(f"{'ms/step':>8} {'calls/step':>10} {'avg us':>9} {'%':>6}  kernel")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:30]:
        t = sum(v)
        print(f"{t / 1e6 / steps:8.3f} {len(v) / steps:10.1f} {t / len(v) / 1e3:9.1f} "
              f"{100 * t / tot:6.2f}  {name[:120]}")


def db(path, steps):
    """Per-kernel stats straight from a rocpd SQLite database (rocprofv3's default output)."""
    import sqlite3

    agg = collections.defaultdict(list)
    for name, d in sqlite3.connect(path).execute("select name, duration from kernels"):
        agg[name].append(int(d))
    tot = sum(sum(v) for v in agg.values())
    print(f"kernel time per step: {tot / 1e6 / steps:.3f} ms over {steps} steps (incl. warm-up/setup kernels)")
    print(f"{'ms/step':>8} {'calls/step':>10} {'avg us':>9} {'%':>6}  kernel")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:30]:
        t = sum(v)
        print(f"{t / 1e6 / steps:8.3f} {len(v) / steps:10.1f} {t / len(v) / 1e3:9.1f} "
              f"{100 * t / tot:6.2f}  {name[:120]}")


def pmc(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            n = r["Kernel_Name"]
            if "sdml" not in n and "Cijk" not in n:  # (hipBLASLt's GEMMs kept for A/B passes)
                continue
            key = n.replace("sdml::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        print(f"== {k}  (dispatch {sorted(dur[k])[len(dur[k]) // 2]:.1f} us median, profiled)")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:.4g}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':28s} {100 * m[c] / wc:.1f} %")
        if "FETCH_SIZE" in m:
            print(f"   {'HBM bytes read (2 x FETCH_SIZE KB)':28s} {2 * m['FETCH_SIZE'] / 1e3:.1f} MB")


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], int(sys.argv[3]))
    elif sys.argv[1] == "db":
        db(sys.argv[2], int(sys.argv[3]))
    elif sys.argv[1] == "trace":
        trace(sys.argv[2], int(sys.argv[3]))
    else:
        pmc(sys.argv[2:])
