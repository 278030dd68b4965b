"""Per-kernel resource usage of librfrt's own kernels (VGPRs, SGPRs, scratch, dynamic stack, LDS,
occupancy), from the compiler's resource-usage remarks for the code objects the library is built from.

    python tools/kernel_resources.py [--out profiles/rNN_kernel_resources] [source.hip ...]

With --out, also writes <out>.json (every remark field per kernel) and <out>.md (the table).

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


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                           text=True, timeout=60)
        out = r.stdout.splitlines()
        if len(out) == len(names):
            return out
    except (OSError, subprocess.SubprocessError):
        pass
    return names


def main(argv):
    import json
    out = None
    if argv[:1] == ["--out"]:
        out, argv = argv[1], argv[2:]
    srcs = argv or sorted(glob.glob(os.path.join(B.CSRC, "*.hip")))
    table = []
    for src in srcs:
        rows = resources(src)
        for r, d in zip(rows, demangle([r["name"] for r in rows])):
            r["source"] = os.path.basename(src)
            r["demangled"] = d
            table.append(r)
            print(f"{r['source']:14s} VGPR {r.get('VGPRs', '?'):>4s} SGPR {r.get('TotalSGPRs', '?'):>3s} "
                  f"spill {r.get('VGPRs Spill', '?'):>3s} "
                  f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>5s} dynstack {r.get('Dynamic Stack', '?'):5s} "
                  f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2s} LDS {r.get('LDS Size [bytes/block]', '?'):>6s}  "
                  f"{d[:100]}")
    if out:
        with open(out + ".json", "w") as f:
            json.dump({"cflags": B.CFLAGS, "kernels": table}, f, indent=1)
        with open(out + ".md", "w") as f:
            f.write("# Kernel resources (compiler remarks, `python tools/kernel_resources.py --out ...`)\n\n")
            f.write("Flags: `" + " ".join(B.CFLAGS) + "`\n\n")
            f.write("| source | kernel | VGPRs | VGPR spills | AGPRs | SGPRs | scratch B/lane | dyn. stack | LDS B/block "
                    "| waves/SIMD |\n")
            f.write("|---|---|---|---|---|---|---|---|---|---|\n")
            for r in table:
                f.write(f"| {r['source']} | `{r['demangled'][:120]}` | {r.get('VGPRs', '?')} | {r.get('VGPRs Spill', '?')} | "
                        f"{r.get('AGPRs', '?')} | {r.get('TotalSGPRs', '?')} | {r.get('ScratchSize [bytes/lane]', '?')} | "
                        f"{r.get('Dynamic Stack', '?')} | {r.get('LDS Size [bytes/block]', '?')} | "
                        f"{r.get('Occupancy [waves/SIMD]', '?')} |\n")


if __name__ == "__main__":
    main(sys.argv[1:])
