"""HBM bytes per self-attention launch from the two PMC passes of scripts/pmc_attn.sh (kbench launches) or, with
--bench, of scripts/pmc_bench.sh (the bench's own clip; also the persistent GEMMs by epilogue).
FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced read (MI355X_MICROARCH.md §HBM), so it is doubled.  Infinity-Cache hits are included.
usage: python scripts/pmc_traffic.py <gpurun_out dir> <out.json>"""
import csv
import json
import statistics
import sys


def _grid(r):
    return int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)


def per_launch(path, kernel="attn_fwd"):
    vals, name = [], None
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and _grid(r) >= 512 * 84:
                vals.append(float(r["Counter_Value"]))
                name = r["Kernel_Name"]
    return statistics.mean(vals), len(vals), name


def gemm_sizes(path):
    """per persistent-GEMM epilogue: the counter values of the full-size launches (the top cluster), in KiB"""
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if "gemm_s8_kernel<" in n:
                out.setdefault(n.split("gemm_s8_kernel<")[1][0], []).append(float(r["Counter_Value"]))
    return out


def main(d, out, bench=False):
    pre = "pmcb" if bench else "pmc"
    f, nf, name = per_launch(f"{d}/{pre}_FETCH_SIZE/run_counter_collection.csv")
    w, nw, _ = per_launch(f"{d}/{pre}_WRITE_SIZE/run_counter_collection.csv")
    L, H, D = 21504, 12, 128
    algo = 4 * 3 * L * H * D * 2
    res = {"kernel": name, "launches": [nf, nw], "fetch_size_kib_raw": round(f, 1), "write_size_kib": round(w, 1),
           "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024), "algorithmic_bytes_per_launch": algo,
           "note": "FETCH_SIZE x2 (gfx950 correction); Infinity-Cache hits are counted, so K/V re-reads that "
                   "miss the per-XCD L2 appear here even when served on-die"}
    res["traffic_over_algorithmic"] = round(res["hbm_bytes_per_launch"] / algo, 2)
    if bench:
        res["source"] = ("scripts/pmc_bench.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                         "bench.py's own clip (2 sampling steps, 60 self-attention launches at B=3, L=21504)")
        fs = gemm_sizes(f"{d}/{pre}_FETCH_SIZE/run_counter_collection.csv")
        ws = gemm_sizes(f"{d}/{pre}_WRITE_SIZE/run_counter_collection.csv")
        g = {}
        for epi in sorted(fs):
            big_f = sorted(fs[epi])[len(fs[epi]) // 2:]  # the upper half: the DiT-layer launches
            big_w = sorted(ws.get(epi, [0.0]))[len(ws.get(epi, [0.0])) // 2:]
            g[f"epilogue_{epi}"] = {"launches": len(fs[epi]),
                                    "fetch_bytes_median_upper_half": int(2 * statistics.median(big_f) * 1024),
                                    "write_bytes_median_upper_half": int(statistics.median(big_w) * 1024)}
        res["gemm_s8"] = g
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    a = [x for x in sys.argv[1:] if x != "--bench"]
    main(a[0], a[1], bench="--bench" in sys.argv)
