"""Per-dispatch table of a rocprofv3 --pmc run: duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs /
wall), MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 256 CUs x 4 SIMDs)) and the raw
counters.  usage: python scripts/pmc_table.py <dir with run_counter_collection.csv> [min_us]"""
import collections
import csv
import os
import sys


def main(d, min_us=50.0):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    trace = {}
    tp = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tp):
        trace = {r["Dispatch_Id"]: r for r in csv.DictReader(open(tp))}
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in rows:
        k = r["Dispatch_Id"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    for k in sorted(agg, key=int):
        a = agg[k]
        t = trace.get(k)
        dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) if t else 0
        if dur < min_us * 1e3:
            continue
        out = [k, names[k][:70], "us=%.0f" % (dur / 1e3)]
        if "GRBM_GUI_ACTIVE" in a and dur:
            clk = a["GRBM_GUI_ACTIVE"] / 8 / dur
            out.append("GHz=%.2f" % clk)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
                out.append("mfma=%.3f" % (a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)))
        if "SQ_WAVE_CYCLES" in a:
            wc = a["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in a:
                    out.append("%s=%.2f" % (c[3:], a[c] / wc))
        for c, v in a.items():
            if c not in ("GRBM_GUI_ACTIVE",):
                out.append("%s=%.4g" % (c, v))
        print(" ".join(out))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 50.0)
