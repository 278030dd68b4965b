"""Summarize a tools/gpu.sh stats + pmc run (gpurun_out/prof_<TAG>/{stats,p1..}) into profiles/:

  <tag>_kernel_stats.csv   rocprofv3 --stats of the trace pass (average duration per kernel)
  <tag>_pmc.json           per-launch means of every PMC counter for the kernels of the hot path,
                           HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, KB -> B; MI355X_MICROARCH.md
                           'HBM': gfx950 reports half of the bytes of wide reads), L2 hit rate
  traffic_legs.json        the same HBM bytes per launch keyed by kernel, read by bench.py to fill
                           each leg's roofline "traffic" (a property of code + input, like the
                           FETCH/WRITE of the K2 kernel in traffic_k2.json)
  traffic_k2.json, k2_sq_counters.json   refreshed for the K2 kernel

    python tools/summarize_r2.py <tag> [config note]
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {  # short name -> substring of the demangled rocprofv3 name
    "k_trace_bf<3>": "k_trace_bf<3, false>",
    "k_trace_bvh<5>": "k_trace_bvh<5>",
    "k_traj<false>": "k_traj<false>",
    "k_traj<true>": "k_traj<true>",
    "k_replay<false>": "k_replay<false",
    "k_replay<true>": "k_replay<true",
    "k_win": "k_win(",
    "k_cells": "k_cells(",
    "k_cols": "k_cols(",
    "k_power": "k_power(",
    "k_power_small<1>": "k_power_small<1>(",
    "k_power_small<8>": "k_power_small<8>(",
    "k_power_small<16,32>": "k_power_small<16, 32>(",
    "k_fill_received": "k_fill_received(",
}


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    for k, sub in KERNELS.items():
        if sub in n:
            return k
    return None


def counters(base):
    """{short kernel: {counter: mean per dispatch}} over every pass directory.  k_fill_received
    serves both the K2 and the K4 step (different sizes): each of its dispatches is attributed to
    the trace kernel dispatched right after it on the same pass ("k_fill_received@k2" before
    k_trace_bf<3>, "@k4" before k_trace_bvh<5>), so each leg's traffic adds its own fill."""
    acc = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(base, "p*", "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        names = {int(r["Dispatch_Id"]): short(r["Kernel_Name"]) for r in rows}
        for r in rows:
            k = short(r["Kernel_Name"])
            if k is None:
                continue
            if k == "k_fill_received":
                nxt = names.get(int(r["Dispatch_Id"]) + 1)
                k = {"k_trace_bf<3>": "k_fill_received@k2", "k_trace_bvh<5>": "k_fill_received@k4"}.get(nxt, k)
            d = acc[k][r["Counter_Name"]]
            key = (f, r["Dispatch_Id"])
            d[key] = d.get(key, 0.0) + float(r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} | {"dispatches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


def durations(base):
    out = {}
    for f in glob.glob(os.path.join(base, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            if k:
                out[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def main(tag, note=""):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = glob.glob(os.path.join(base, "stats", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    pmc, dur = counters(base), durations(base)
    out = {"tag": tag, "note": note,
           "how": "rocprofv3 --kernel-trace --stats pass + one --pmc pass per counter group (tools/gpu.sh stats, pmc); "
                  "means per dispatch; HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) KB x 1024",
           "kernels": {}}
    for k in sorted(set(pmc) | set(dur)):
        c = pmc.get(k, {})
        e = {"avg_us": dur.get(k, {}).get("avg_us"), "calls": dur.get(k, {}).get("calls"), "counters": c}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            if e["avg_us"]:
                e["hbm_gbs"] = e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e-6) / 1e9
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "SQ_INSTS_VALU" in c and e["avg_us"]:
            e["valu_frac_of_issue_peak"] = c["SQ_INSTS_VALU"] / (e["avg_us"] * 1e-6) / (1024 * 2.4e9 / 2)
        out["kernels"][k] = e
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w"), indent=1)
    legs = {k: {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "l2_hit_rate": v.get("l2_hit_rate"),
                "avg_us": v["avg_us"], "source": f"profiles/{tag}_pmc.json", "note": note}
            for k, v in out["kernels"].items() if "hbm_bytes_per_launch" in v}
    # a K4 step is the coalesced NaN / 0 fill of received and row_mask, then the trace kernel (which
    # stores only the received rows): the leg's traffic is both launches' bytes
    for trace, fill in (("k_trace_bvh<5>", "k_fill_received@k4"), ("k_trace_bf<3>", "k_fill_received@k2")):
        if trace in legs and fill in legs:
            t, f = legs[trace], legs[fill]
            t["trace_kernel_bytes_per_launch"] = t["hbm_bytes_per_launch"]
            t["fill_bytes_per_launch"] = f["hbm_bytes_per_launch"]
            t["hbm_bytes_per_launch"] += f["hbm_bytes_per_launch"]
            t["note"] = (t["note"] + "; " if t["note"] else "") + f"{trace} + its {fill}"
    json.dump(legs, open(os.path.join(ROOT, "profiles", "traffic_legs.json"), "w"), indent=1)
    k2 = out["kernels"].get("k_trace_bf<3>", {})
    if "hbm_bytes_per_launch" in k2:
        c = k2["counters"]
        fill = out["kernels"].get("k_fill_received@k2", {})
        fb = fill.get("hbm_bytes_per_launch")
        # the K2 step's span (bench roofline: HIP events from the fill's start to the trace kernel's
        # end) covers both launches, so its traffic is both launches' bytes
        json.dump({"kernel": "k_fill_received + k_trace_bf<3, false>", "rays": 1_000_000, "bounces": 3,
                   "how": out["how"], "fetch_size_kb_per_launch": c["FETCH_SIZE"],
                   "write_size_kb_per_launch": c["WRITE_SIZE"],
                   "trace_kernel_bytes_per_launch": k2["hbm_bytes_per_launch"],
                   "fill_bytes_per_launch": fb,
                   "fill_counters": fill.get("counters"),
                   "hbm_bytes_per_launch": k2["hbm_bytes_per_launch"] + (fb or 0.0),
                   "algorithmic_bytes_per_launch": 1_000_000 * (24 * 4 + 4), "tag": tag},
                  open(os.path.join(ROOT, "profiles", "traffic_k2.json"), "w"), indent=1)
        if "SQ_INSTS_VALU" in c:
            json.dump(dict(c, source=f"profiles/{tag}_pmc.json (k_trace_bf<3, false>, tools/gpu.sh pmc)"),
                      open(os.path.join(ROOT, "profiles", "k2_sq_counters.json"), "w"), indent=1)
    for k, v in out["kernels"].items():
        print(f"{k:18s} avg {v['avg_us'] or 0:9.1f} us  HBM {v.get('hbm_bytes_per_launch', 0) / 1e6:8.2f} MB  "
              f"L2 hit {v.get('l2_hit_rate') or 0:.3f}  VALU {v.get('valu_frac_of_issue_peak') or 0:.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "run", " ".join(sys.argv[2:]))
