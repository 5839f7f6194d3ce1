#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (VGPRs, AGPRs, scratch, occupancy, LDS), from the
compiler's -Rpass-analysis=kernel-resource-usage remarks, with tools/build.py's flags for that file.
    python tools/kres.py quantizedmha_amd/csrc/qmha_fa_int8.hip [-D...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools import build  # noqa: E402


def main():
    src = os.path.abspath(sys.argv[1])
    extra = sys.argv[2:]
    flags = build.COMMON_FLAGS + build.FILE_FLAGS.get(os.path.basename(src), []) + extra
    cmd = [build.HIPCC] + flags + ["-I", os.path.join(ROOT, "include"), "-I", build.CSRC, "-c", "-x", "hip", src, "-o",
                                   "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    cur = None
    rows = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        msg = m.group(1).strip()
        if msg.startswith("Function Name:"):
            cur = {"name": msg.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in msg:
            k, v = msg.split(":", 1)
            cur[k.strip()] = v.strip()
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-3000:])
        sys.exit(r.returncode)
    for c in rows:
        name = subprocess.run(["c++filt"], input=c["name"], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name).replace("qmha::", "")
        print(f"{name:60s} vgpr {c.get('VGPRs', '?'):>4s} agpr {c.get('AGPRs', '?'):>4s} scratch "
              f"{c.get('ScratchSize [bytes/lane]', '?'):>5s} occ {c.get('Occupancy [waves/SIMD]', '?'):>2s} "
              f"lds {c.get('LDS Size [bytes/block]', '?')}")


if __name__ == "__main__":
    main()
