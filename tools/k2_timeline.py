"""Kernel timeline of the last K2 bench steps from a rocprofv3 --kernel-trace CSV
(python bench.py --legs k2 ...): per step, every kernel's duration and the gaps between them.

    python tools/k2_timeline.py gpurun_out/<dir> [steps]
"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_trace_bf" in r["Kernel_Name"]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for a, b in zip(starts[-n - 1:-1], starts[-n:]):
    t0 = int(rows[a]["Start_Timestamp"])
    prev, out = t0, []
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = r["Kernel_Name"]
        j = nm.find("k_")
        nm = "rocprim" if "rocprim" in nm else ("fill" if "fill" in nm else (
            nm[j:j + 18].split("(")[0] if j >= 0 else nm[:18]))
        out.append((f"[gap {(s - prev) / 1e3:.1f}] " if s - prev > 500 else "") + f"{nm}:{(e - s) / 1e3:.1f}")
        prev = e
    print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us:", " ".join(out))
