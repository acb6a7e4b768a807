"""Kernel-trace gaps: read a rocprofv3 `--kernel-trace --output-format csv`
kernel_trace.csv and report, for the last N back-to-back calls of a repeated
launch sequence, each kernel's duration and the idle time between one
kernel's end and the next kernel's start (the GPU-idle share a host-bound
call would show).  Usage:

    python tools/trace_gaps.py <kernel_trace.csv> --per-call 3 --calls 20 [--json out.json]
"""
import argparse
import csv
import json
import statistics


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("dctae::", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--per-call", type=int, required=True, help="kernels per call")
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--match", action="append", default=[], help="only kernels whose name contains one of these")
    ap.add_argument("--first", type=int, default=None,
                    help="take the calls starting at this call index (default: the last --calls calls)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    rows = [r for r in load(args.csv) if not args.match or any(m in r[2] for m in args.match)]
    n = args.per_call * args.calls
    rows = rows[-n:] if args.first is None else rows[args.per_call * args.first:args.per_call * args.first + n]
    per_kernel, gaps_in, gaps_between, spans = {}, [], [], []
    for c in range(args.calls):
        call = rows[c * args.per_call:(c + 1) * args.per_call]
        for i, (s, e, nm) in enumerate(call):
            per_kernel.setdefault((i, short(nm)), []).append((e - s) / 1e3)
            if i:
                gaps_in.append((s - call[i - 1][1]) / 1e3)
        spans.append((call[-1][1] - call[0][0]) / 1e3)
        if c:
            gaps_between.append((call[0][0] - rows[c * args.per_call - 1][1]) / 1e3)
    busy = sum(statistics.mean(v) for v in per_kernel.values())
    period = (rows[-1][1] - rows[0][0]) / 1e3 / args.calls
    out = {
        "calls": args.calls,
        "kernels_us": {f"{i}:{nm}": round(statistics.mean(v), 2) for (i, nm), v in sorted(per_kernel.items())},
        "busy_us_per_call": round(busy, 2),
        "gap_inside_call_us_mean": round(statistics.mean(gaps_in), 2) if gaps_in else None,
        "gap_between_calls_us_mean": round(statistics.mean(gaps_between), 2) if gaps_between else None,
        "gap_between_calls_us_max": round(max(gaps_between), 2) if gaps_between else None,
        "span_us_per_call": round(statistics.mean(spans), 2),
        "period_us_per_call": round(period, 2),
        "gpu_idle_share": round(1 - busy / period, 4),
    }
    print(json.dumps(out, indent=1))
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
