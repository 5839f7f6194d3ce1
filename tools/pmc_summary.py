#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel (sum over dispatches / dispatch count).

usage: python tools/pmc_summary.py <dir-with-pmc*/run_counter_collection.csv> [--kernel substr]
       [--json-out profiles/rNN/pmc_<variant>.json --shape B H N d]
HBM traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE (kB) reports half
of a wide coalesced stream's bytes on gfx950 -> bytes_read = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (kB) is exact for 16-B/lane streaming stores -> bytes_written = WRITE_SIZE * 1024.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            per[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[(k, row["Counter_Name"])].add((f, row["Dispatch_Id"]))
    out = {}
    for k, ctrs in per.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in ctrs.items()}
    return out


def short(name):
    return name.split("(")[0].replace("void ", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="qmha")
    ap.add_argument("--json-out")
    ap.add_argument("--shape", nargs=4, type=int)
    a = ap.parse_args()
    data = load(a.dir)
    res = {}
    for k, c in sorted(data.items()):
        if a.kernel not in k:
            continue
        print(short(k))
        for n in sorted(c):
            print(f"    {n:32s} {c[n]:.6g}")
        der = {}
        if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
            der["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
            der["mfma_insts_per_wave"] = c.get("SQ_INSTS_MFMA", 0) / c["SQ_WAVES"]
        if "FETCH_SIZE" in c:
            der["hbm_read_bytes_per_launch"] = 2 * c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            der["hbm_write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy cycles over all 1024 SIMDs
            der["mfma_busy_pct"] = 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
            der["effective_clock_ghz_x_ms"] = c["GRBM_GUI_ACTIVE"] / 8 / 1e6
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
            der["valu_active_per_wave_cycle"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        for n, v in der.items():
            print(f"  = {n:30s} {v:.6g}")
        res[short(k)] = {"counters": c, "derived": der}
    if a.json_out:
        # the main kernel of the shape's head size: template argument d (mangled ILi<d>E or <d, ...>)
        dd = a.shape[3] if a.shape else None
        main_k = [k for k in res if "fa_" in k and "kernel" in k and
                  (dd is None or f"ILi{dd}E" in k or f"<{dd}," in k)]
        j = {"source": a.dir, "kernels": res}
        if main_k and a.shape:
            d = res[main_k[0]]["derived"]
            if "hbm_read_bytes_per_launch" in d and "hbm_write_bytes_per_launch" in d:
                j["hbm_bytes_per_launch"] = d["hbm_read_bytes_per_launch"] + d["hbm_write_bytes_per_launch"]
            for key in ("mfma_busy_pct", "valu_insts_per_wave"):  # bench.py's roofline.mfma_busy_pct
                if key in d:
                    j[key] = d[key]
            j["shape"] = a.shape
            j["kernel"] = main_k[0]
        os.makedirs(os.path.dirname(a.json_out), exist_ok=True)
        json.dump(j, open(a.json_out, "w"), indent=1)


if __name__ == "__main__":
    main()
