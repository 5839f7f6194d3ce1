#!/bin/bash
# r04q: per-dispatch durations of the single-read per-tensor pre-pass (bench as a sibling measurement
# and as the headline) -- looking for bounded-wait fallbacks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 300 python bench.py --variant fa_tc_int8_pt --steps 25 --warmup 2 --no-siblings --no-cpu-baseline --no-solve-calls --no-refconfig > $O/b_w2.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --variant fa_tc_int8_pt --steps 20 --warmup 20 --no-siblings --no-cpu-baseline --no-solve-calls --no-refconfig > $O/b_w20.json 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("b_w2", "b_w20"):
    j = json.loads(open(f"gpurun_out/r04q/{f}.json").read().strip().splitlines()[-1])
    print(f, j["ms_per_step"], j["roofline"]["main_kernel_ms"], j["roofline"]["prepass_ms"])
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls --no-refconfig > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/trace
python3 - <<'PY'
import csv
rows = [r for r in csv.DictReader(open("gpurun_out/r04q/kernel_trace.csv")) if "pt_quant" in r["Kernel_Name"] or "zero_u32" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:30]) for r in rows]
pq = [x for x, n in d if "pt_quant" in n]
print("pt_quant dispatches", len(pq), "min %.1f max %.1f us" % (min(pq), max(pq)))
print("durations (us):", " ".join("%.0f" % x for x in pq))
PY
