"""Group a rocprofv3 kernel trace (…_kernel_trace.csv) by (kernel, grid, workgroup, LDS) and print calls, mean
and total duration per group, largest total first: separates the shapes one kernel name serves in a clip.
usage: python scripts/trace_shapes.py <run_kernel_trace.csv> [top]"""
import csv
import sys
from collections import defaultdict


def main(path, top=40):
    g = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", r.get("KernelName", ""))
            name = name.replace("(anonymous namespace)::", "")[:70]
            grid = r.get("Grid_Size") or "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            wg = r.get("Workgroup_Size", r.get("Workgroup_Size_X", ""))
            lds = r.get("LDS_Block_Size", r.get("Lds_Size", ""))
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            g[(name, grid, wg, lds)].append(d)
    rows = sorted(g.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for v in g.values())
    print(f"{'kernel':70s} {'grid':>9s} {'wg':>5s} {'calls':>6s} {'mean_us':>9s} {'total_ms':>9s} {'pct':>6s}")
    for (name, grid, wg, lds), v in rows[:top]:
        print(f"{name:70s} {grid:>9s} {wg:>5s} {len(v):6d} {sum(v) / len(v) / 1e3:9.1f} {sum(v) / 1e6:9.1f} "
              f"{100 * sum(v) / tot:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
