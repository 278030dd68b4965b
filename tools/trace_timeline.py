"""Print the kernel timeline after each map's replay kernel from a rocprofv3 --kernel-trace CSV
(the reduce + power stage of tools/cov_variants.py child k3,k5 1).

    python tools/trace_timeline.py gpurun_out/<tag>_trace
"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_replay<" in r["Kernel_Name"]]
for case, a in zip(("k3", "k5"), idx[-2:]):
    t0 = int(rows[a]["End_Timestamp"])
    out, e = [], t0
    for r in rows[a + 1:a + 60]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = r["Kernel_Name"]
        j = n.find("k_")
        nm = "rocprim" if "rocprim" in n else ("fill" if "fill" in n else (n[j:j + 16] if j >= 0 else n[:16]))
        out.append(f"{nm.split('(')[0]}:{(e - s) / 1e3:.0f}")
        if "k_power(" in n:
            break
    print(case, f"reduce+power {(e - t0) / 1e3:.0f} us:", " ".join(out))
