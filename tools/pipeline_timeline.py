"""The two-stream timeline of one pipelined C5 run (rthx.distributed
trace_bands_row_sharded, emulated rank) from a rocprofv3 --kernel-trace CSV
of `tools/bench_c5_bands.py --emulate-world W --pipeline --ranks q --reps 1`.

That command launches, in order: the peers' pieces of the rank's band
(traced beforehand), then the overlapped pipeline (one warm-up run, one timed
run) and the sequential one (idem).  The timed overlapped run is the
`--run`-th group of `--traces` trace_exchange_kernel launches after the
`--skip` peer traces.  Prints every kernel of that run by queue (HIP stream)
with start / end relative to its first trace kernel, and the critical path
(first trace kernel start -> last kernel end of the run).

  python tools/pipeline_timeline.py run_kernel_trace.csv --skip 14 --traces 9
"""
import argparse
import csv


def short(name):
    for k in ("trace_exchange_kernel", "row_scan_kernel", "csr_pack_kernel", "k_shard_scan", "k_shard_copy",
              "copyBuffer", "fillBuffer", "FillFunctor", "direct_copy", "elementwise"):
        if k in name:
            return k
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, default=14, help="trace kernels before the pipeline runs (peer pieces)")
    ap.add_argument("--traces", type=int, default=9, help="trace kernels per pipeline run")
    ap.add_argument("--run", type=int, default=1, help="0-based pipeline run after the skipped traces (1: the timed overlapped run)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tr = [i for i, r in enumerate(rows) if "trace_exchange_kernel" in r["Kernel_Name"]]
    first = tr[a.skip + a.run * a.traces]
    nxt = a.skip + (a.run + 1) * a.traces
    end_idx = tr[nxt] if nxt < len(tr) else len(rows)
    run = rows[first:end_idx]
    # the run ends with its last merge kernel (k_shard_copy), or its last kernel
    last = max(i for i, r in enumerate(run) if "k_shard_copy" in r["Kernel_Name"]) if any(
        "k_shard_copy" in r["Kernel_Name"] for r in run) else len(run) - 1
    run = run[:last + 1]
    t0 = int(run[0]["Start_Timestamp"])
    busy = {}
    print(f"{'queue':>5} {'kernel':24s} {'start ms':>9} {'end ms':>9} {'dur ms':>8}")
    for r in run:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
        q = r["Queue_Id"]
        busy.setdefault(q, 0.0)
        busy[q] += e - s
        if e - s >= 0.05 or "shard" in r["Kernel_Name"] or "trace" in r["Kernel_Name"]:
            print(f"{q:>5} {short(r['Kernel_Name']):24s} {s:9.3f} {e:9.3f} {e - s:8.3f}")
    crit = (max(int(r["End_Timestamp"]) for r in run) - t0) / 1e6
    traces = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in run
                 if "trace_exchange_kernel" in r["Kernel_Name"])
    print(f"critical path (first trace kernel -> last kernel of the run): {crit:.2f} ms; trace kernels {traces:.2f} ms; "
          "busy ms per queue: " + ", ".join(f"{q}: {v:.2f}" for q, v in busy.items()))


if __name__ == "__main__":
    main()
