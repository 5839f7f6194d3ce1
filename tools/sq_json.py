#!/usr/bin/env python3
"""Convert a tools/pmc_sq.sh summary (gpurun_out/<tag>/summary.txt) into the JSON bench.py cites
for the main kernel's MFMA-busy % (profiles/<round>/pmc_sq_<variant>.json).

    python tools/sq_json.py <summary.txt> <out.json> [--shape B H N d] [--kernel-substr pipe_kernelILi64]
"""
import argparse
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("out")
    ap.add_argument("--shape", type=int, nargs=4, default=[16, 16, 4096, 64])
    ap.add_argument("--kernel-substr", default="pipe_kernelILi64")
    a = ap.parse_args()
    out = {"source": a.summary, "shape": a.shape, "kernels": {}}
    for block in re.split(r"\n(?=\S)", open(a.summary).read()):
        lines = block.strip().split("\n")
        vals = {}
        for line in lines[1:]:
            m = re.match(r"\s*=?\s*(\S+)\s+(\S+)$", line)
            if m:
                try:
                    vals[m.group(1)] = float(m.group(2))
                except ValueError:
                    pass
        if vals:
            out["kernels"][lines[0].strip()] = vals
    k = next(n for n in out["kernels"] if a.kernel_substr in n)
    out["kernel"] = k
    out["mfma_busy_pct"] = out["kernels"][k].get("mfma_busy_pct")
    out["valu_insts_per_wave"] = out["kernels"][k].get("valu_insts_per_wave")
    json.dump(out, open(a.out, "w"), indent=1)
    print(k, out["mfma_busy_pct"])


if __name__ == "__main__":
    main()
