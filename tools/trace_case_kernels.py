"""Average kernel durations per coverage case from a rocprofv3 kernel trace of tools/cov_profile.py.

Usage: python tools/trace_case_kernels.py <trace dir> [kernel substrings...]
A dispatch belongs to the case of the last trajectory kernel before it (k_traj<true> / k_traj_split:
K5, BVH; k_traj<false> / k_traj_lds_split: K3), and to the one-GPU map or a rank plan by the
trajectory kernel's form (k_traj<...>: the whole map; the split forms: a rank's share)."""
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    keys = sys.argv[2:] or ["k_traj", "k_cols", "k_cells", "k_win", "k_replay<", "k_send_runs", "k_merge_lockstep",
                            "k_owner_runs", "k_terms", "k_cell_ranges", "k_power_small", "k_power("]
    f = (glob.glob(f"{d}/**/k_kernel_trace.csv", recursive=True) + glob.glob(f"{d}/k_kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    tag, out = None, {}
    for r in rows:
        n = r["Kernel_Name"]
        if "k_traj<true>" in n:
            tag = "k5 map"
        elif "k_traj_split" in n:
            tag = "k5 rank"
        elif "k_traj<false>" in n:
            tag = "k3 map"
        elif "k_traj_lds_split" in n:
            tag = "k3 rank"
        for k in keys:
            if k in n and tag:
                out.setdefault(tag, {}).setdefault(k.rstrip("(<"), []).append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(json.dumps({t: {k: round(sum(v) / len(v), 1) for k, v in ks.items()} for t, ks in out.items()}))


if __name__ == "__main__":
    main()
