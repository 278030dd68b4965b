"""Summarize a tools/profile.sh run (gpurun_out/prof_<TAG>/{trace,fetch,write}) into profiles/:
<tag>_kernel_stats.csv (rocprofv3 --stats of the trace pass) and traffic_k2.json (per-launch HBM
bytes of the K2 trace kernel: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md 'HBM' gfx950 note)."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_trace_bf<3, false>"


def per_kernel(path):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            d = out.setdefault(k, {})
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: {"calls": len(v), "mean_kb": sum(v.values()) / len(v)} for k, v in out.items()}


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = glob.glob(os.path.join(base, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    fetch, write = per_kernel(os.path.join(base, "fetch")), per_kernel(os.path.join(base, "write"))
    name = next((k for k in fetch if KERNEL in k.replace("(anonymous namespace)::", "")), None)
    if name is None:
        sys.exit(f"no {KERNEL} dispatches in {base}/fetch")
    f_kb, w_kb = fetch[name]["mean_kb"], write[name]["mean_kb"]
    out = {
        "kernel": name, "rays": 1_000_000, "bounces": 3,
        "how": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (tools/profile.sh) over bench.py; "
               "KB units; FETCH_SIZE doubled per MI355X_MICROARCH.md 'HBM' (gfx950 reports half of wide reads)",
        "fetch_size_kb_per_launch": f_kb, "write_size_kb_per_launch": w_kb,
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
        "algorithmic_bytes_per_launch": 1_000_000 * (24 * 4 + 4),
        "all_kernels": {"FETCH_SIZE": fetch, "WRITE_SIZE": write}, "tag": tag,
    }
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_k2.json"), "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("kernel", "hbm_bytes_per_launch", "algorithmic_bytes_per_launch")}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "run")
