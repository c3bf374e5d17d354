"""Summarise rocprofv3 CSV output (kernel stats and --pmc counters).

Usage:
  python tools/pmc_summary.py stats <dir>                  # kernel_stats.csv table
  python tools/pmc_summary.py pmc <dir> [<dir> ...]        # per-kernel counter means
  python tools/pmc_summary.py traffic <fetch_dir> <write_dir> <out.json>

`traffic` applies the gfx950 corrections of MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reads 1/2 of the bytes of
wide (16 B/lane) coalesced streaming reads.  The correction factor is
recorded next to the raw numbers; for the trace kernel the reads are small
L2-resident gathers, so the raw FETCH_SIZE is reported as the lower bound and
the 2x-corrected value as the upper bound.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(pattern_dir, suffix):
    files = glob.glob(os.path.join(pattern_dir, "**", f"*{suffix}"), recursive=True)
    out = []
    for f in files:
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out, files


def short(name):
    n = name.split("(")[0]
    for key in ("trace_exchange_kernel", "row_scan_kernel", "csr_pack_kernel"):
        if key in n:
            return key + ("" if "trace" not in key else n[n.find("<"):] if "<" in n else "")
    return n[:80]


def stats(d):
    rows, files = _rows(d, "kernel_stats.csv")
    res = []
    for r in rows:
        res.append({
            "name": short(r.get("Name", "")),
            "calls": int(r.get("Calls", 0)),
            "total_ns": float(r.get("TotalDurationNs", 0)),
            "avg_ns": float(r.get("AverageNs", 0)),
            "min_ns": float(r.get("MinNs", 0)),
            "max_ns": float(r.get("MaxNs", 0)),
            "pct": float(r.get("Percentage", 0)),
        })
    return res, files


def pmc(d):
    rows, files = _rows(d, "counter_collection.csv")
    acc = defaultdict(lambda: defaultdict(list))
    for r in rows:
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in cs.items()}
    return out, files


def main():
    mode = sys.argv[1]
    if mode == "stats":
        res, files = stats(sys.argv[2])
        print(json.dumps({"files": files, "kernels": res}, indent=1))
    elif mode == "pmc":
        merged = {}
        for d in sys.argv[2:]:
            o, _ = pmc(d)
            for k, v in o.items():
                merged.setdefault(k, {}).update(v)
        print(json.dumps(merged, indent=1))
    elif mode == "traffic":
        f, _ = pmc(sys.argv[2])
        w, _ = pmc(sys.argv[3])
        key = next((k for k in f if "trace_exchange_kernel" in k), None)
        fetch_kib = f[key]["FETCH_SIZE"]["mean"]
        wkey = next((k for k in w if "trace_exchange_kernel" in k), None)
        write_kib = w[wkey]["WRITE_SIZE"]["mean"]
        out = {
            "kernel": key,
            "fetch_kib_raw": fetch_kib,
            "write_kib_raw": write_kib,
            "hbm_bytes_per_launch": (fetch_kib + write_kib) * 1024.0,
            "hbm_bytes_per_launch_fetch_x2": (2 * fetch_kib + write_kib) * 1024.0,
            "note": "FETCH_SIZE/WRITE_SIZE in KiB (rocprofv3, gfx950); separate --pmc passes; "
                    "fetch x2 = wide-stream correction of MI355X_MICROARCH.md §HBM (upper bound here)",
            "others": {k: v for k, v in f.items() if k != key},
        }
        with open(sys.argv[4], "w") as fh:
            json.dump(out, fh, indent=1)
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
