"""GPU idle time inside each DiT forward of a rocprofv3 kernel trace.

A forward starts at its `timestep_embed_kernel` dispatch and ends at the last kernel that finishes before the
next forward's; busy = the union of the kernel intervals (every stream), idle = span - busy.  Idle time inside a
forward is what host launch gaps (or waits between streams) cost; it is the ceiling of what a HIP graph of the
forward could recover.  usage: python scripts/gap_analysis.py <kernel_trace.csv> [--skip N]"""
import csv
import json
import sys


def main(path, skip=2):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, (_, _, n) in enumerate(rows) if "timestep_embed_kernel" in n]
    out = []
    for j, i0 in enumerate(starts):
        i1 = starts[j + 1] if j + 1 < len(starts) else len(rows)
        ks = rows[i0:i1]
        t0, t1 = ks[0][0], max(e for _, e, _ in ks)
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        for s, e, _ in ks:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        gaps.sort(reverse=True)
        out.append({"forward": j, "kernels": len(ks), "span_ms": round((t1 - t0) / 1e6, 3),
                    "busy_ms": round(busy / 1e6, 3), "idle_ms": round((t1 - t0 - busy) / 1e6, 3),
                    "idle_frac": round((t1 - t0 - busy) / (t1 - t0), 4), "gaps_over_20us": sum(g > 20000 for g in gaps),
                    "largest_gaps_us": [round(g / 1e3, 1) for g in gaps[:5]]})
    for r in out:
        print(json.dumps(r))
    kept = out[skip:] or out
    print(json.dumps({"summary": "mean over forwards %d.." % skip,
                      "span_ms": round(sum(r["span_ms"] for r in kept) / len(kept), 3),
                      "idle_ms": round(sum(r["idle_ms"] for r in kept) / len(kept), 3),
                      "idle_frac": round(sum(r["idle_frac"] for r in kept) / len(kept), 4)}))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[a.index("--skip") + 1]) if "--skip" in a else 2)
