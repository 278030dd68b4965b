"""Per-kernel resource usage of librfrt's own kernels (VGPRs, scratch, dynamic stack, occupancy).

    python tools/kernel_resources.py [source.hip ...]

Compiles each source with the library's flags plus -Rpass-analysis=kernel-resource-usage and
prints one line per kernel of ours (library kernels from rocPRIM/hipCUB are skipped).  A kernel
with "dynamic stack" or a scratch size it cannot bound would read and write per-lane memory the
runtime sizes by default -- the first thing to rule out when results depend on what ran before.
"""
import glob
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from rf_ray_tracing_warp_amd import build as B  # noqa: E402


def resources(src):
    cmd = [B.hipcc(), "-c", src, "-o", os.devnull] + B.CFLAGS + ["-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            name = txt.split(":", 1)[1].strip()
            cur = {"name": name} if ("rocprim" not in name and "hipcub" not in name) else None
            if cur is not None:
                rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def main(argv):
    srcs = argv or sorted(glob.glob(os.path.join(B.CSRC, "*.hip")))
    for src in srcs:
        for r in resources(src):
            print(f"{os.path.basename(src):14s} VGPR {r.get('VGPRs', '?'):>4s} AGPR {r.get('AGPRs', '?'):>3s} "
                  f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>5s} dynstack {r.get('Dynamic Stack', '?'):5s} "
                  f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2s} LDS {r.get('LDS Size [bytes/block]', '?'):>6s}  "
                  f"{r['name'][:90]}")


if __name__ == "__main__":
    main(sys.argv[1:])
