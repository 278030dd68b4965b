"""Compact kernel timeline of the last rank-pass (from its k_traj launch) in a rocprofv3
--kernel-trace CSV of tools/cov_profile.py (SHARDS=8), with gaps.

    python tools/rank_timeline.py gpurun_out/<dir> [case-index]
"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_traj" in r["Kernel_Name"]]
a = starts[-1]
end = len(rows)
t0 = int(rows[a]["Start_Timestamp"])
prev = t0
out = []
for r in rows[a:end]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"]
    j = n.find("k_")
    nm = "rocprim" if "rocprim" in n else ("fill" if "fill" in n else ("copy" if "copyBuffer" in n else (
        n[j:j + 16].split("(")[0] if j >= 0 else n[:16])))
    g = (s - prev) / 1e3
    out.append((f"[gap {g:.0f}] " if g > 3 else "") + f"{nm}:{(e - s) / 1e3:.0f}")
    prev = e
print(f"rank pass {(prev - t0) / 1e3:.0f} us:", " ".join(out))
