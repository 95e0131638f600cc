#!/usr/bin/env python3
"""Summarises a scripts/profile.sh output directory into profiles/<round>/ (kernel stats + per-launch PMC means).

Usage: python scripts/summarize_profile.py gpurun_out/prof profiles/r01 [--tag cfg2_k21_q10_global]
           [--traffic-key cfg2_k21_global_reads1000000_ax]
--traffic-key also records the launch's fabric bytes in profiles/traffic.json under that key, where bench.py looks
them up (cfg<N>_k<k>_<mode>_reads<reads per GPU>_<ax|kt|lf>) for the `traffic` field of its roofline.
Fabric bytes (round 4): TCC_EA0_RDREQ x 128 B + WRITE_SIZE, per profiles/r04/counter_calibration.json
(scripts/calibrate_counters.sh): on gfx950 TCC_BUBBLE and TCC_EA0_RDREQ_32B read 0, so FETCH_SIZE = RDREQ x 64 B,
while one RDREQ is issued per 128-B line filled from the fabric for the 16-B/lane stream (exact: FETCH_SIZE reports
half of a known 2 GiB read, MI355X_MICROARCH.md §HBM) and for 16/64/128-B random gathers (one request per line).
FETCH_SIZE (RDREQ x 64 B) is kept as the lower bound. Infinity-Cache hits are counted (L2 -> fabric requests), so
these are upper bounds on HBM bytes for an index that stays MALL-resident.
"""
import collections
import csv
import json
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    opts = dict(zip(sys.argv[3::2], sys.argv[4::2]))
    tag = opts.get("--tag", "default")
    tkey = opts.get("--traffic-key")
    os.makedirs(dst, exist_ok=True)
    out = {"tag": tag}
    st = os.path.join(src, "trace", "trace_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(dst, f"kernel_stats_{tag}.csv"))
        rows = list(csv.DictReader(open(st)))
        out["kernel_stats"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
                               for r in rows if any(t in r["Name"] for t in ("::k_scan<", "::k_scan_kt<", "::k_scan_ax<"))]
    tr = os.path.join(src, "trace", "trace_kernel_trace.csv")
    if os.path.exists(tr):  # steady state: the later half of the scan dispatches (the first ones run on cold caches)
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(tr))
             if any(t in r["Kernel_Name"] for t in ("::k_scan<", "::k_scan_kt<", "::k_scan_ax<"))]
        if d:
            tail = d[len(d) // 2:]
            out["scan_dispatch_ns"] = d
            out["scan_steady_state_avg_ns"] = sum(tail) / len(tail)
    pmc = collections.defaultdict(list)
    meta = {}
    for p in ("fetch", "write", "tcc", "sq", "sq2", "ta", "req"):
        f = os.path.join(src, p, f"{p}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if not any(t in r["Kernel_Name"] for t in ("::k_scan<", "::k_scan_kt<", "::k_scan_ax<")):  # not rocPRIM's scans
                continue
            pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "SGPR_Count",
                                      "Scratch_Size")}
    means = {k: sum(v) / len(v) for k, v in pmc.items()}
    out["k_scan_pmc_mean_per_launch"] = means
    out["k_scan_dispatch"] = meta
    if "FETCH_SIZE" in means:
        out["fabric_read_bytes_per_launch"] = means["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in means:
        out["fabric_write_bytes_per_launch"] = means["WRITE_SIZE"] * 1024
    if "TCC_EA0_RDREQ_sum" in means and "FETCH_SIZE" in means:
        out["check_fetch_equals_rdreq_x64"] = abs(means["TCC_EA0_RDREQ_sum"] * 64 - means["FETCH_SIZE"] * 1024) \
            / max(1.0, means["FETCH_SIZE"] * 1024)
    if "TCC_HIT_sum" in means:
        h, m = means["TCC_HIT_sum"], means.get("TCC_MISS_sum", 0.0)
        out["l2_hit_rate"] = h / max(1.0, h + m)
    if "TCC_EA0_RDREQ_sum" in means:  # calibrated: 128 B per request (profiles/r04/counter_calibration.json)
        out["fabric_read_bytes_calibrated"] = means["TCC_EA0_RDREQ_sum"] * 128.0
        out["fabric_read_bytes_lower_bound"] = means["TCC_EA0_RDREQ_sum"] * 64.0
        if "TCC_BUBBLE_sum" in means:
            out["tcc_bubble"] = means["TCC_BUBBLE_sum"]
            out["tcc_rdreq_32b"] = means.get("TCC_EA0_RDREQ_32B_sum")
    json.dump(out, open(os.path.join(dst, f"pmc_{tag}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))
    if tkey and "fabric_read_bytes_calibrated" in out:
        tp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
        tj = json.load(open(tp)) if os.path.exists(tp) else {}
        wr = out.get("fabric_write_bytes_per_launch", 0.0)
        tj[tkey] = {"fabric_bytes_per_launch": out["fabric_read_bytes_calibrated"] + wr,
                    "fabric_read_bytes_per_launch": out["fabric_read_bytes_calibrated"],
                    "fabric_bytes_lower_bound": out["fabric_read_bytes_lower_bound"] + wr,
                    "write_bytes_per_launch": out.get("fabric_write_bytes_per_launch"),
                    "method": "TCC_EA0_RDREQ x 128 B + WRITE_SIZE (profiles/r04/counter_calibration.json); lower "
                              "bound RDREQ x 64 B (= FETCH_SIZE)",
                    "source": os.path.relpath(os.path.join(dst, f"pmc_{tag}.json"), os.path.join(os.path.dirname(tp))),
                    "l2_hit_rate": out.get("l2_hit_rate"),
                    "scratch_bytes_per_lane": meta.get("Scratch_Size"), "vgpr_count": meta.get("VGPR_Count"),
                    "kernel_steady_state_ns_rocprof": out.get("scan_steady_state_avg_ns")}
        json.dump(tj, open(tp, "w"), indent=1)
    elif tkey and "fabric_read_bytes_per_launch" in out:
        tp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
        tj = json.load(open(tp)) if os.path.exists(tp) else {}
        scratch = None
        if meta.get("Scratch_Size") not in (None, "") and meta.get("Grid_Size") not in (None, ""):
            scratch = float(meta["Scratch_Size"]) * float(meta["Grid_Size"])  # spill bytes per lane x lanes
        tj[tkey] = {"hbm_bytes_per_launch": out["fabric_read_bytes_per_launch"] + out.get("fabric_write_bytes_per_launch", 0.0),
                    "fetch_bytes_per_launch": out["fabric_read_bytes_per_launch"],
                    "write_bytes_per_launch": out.get("fabric_write_bytes_per_launch"),
                    "scratch_write_bytes_per_launch": scratch,
                    "scratch_bytes_per_lane": meta.get("Scratch_Size"), "vgpr_count": meta.get("VGPR_Count"),
                    "note": "FETCH_SIZE+WRITE_SIZE (KiB x 1024) per scan launch; L2->fabric bytes incl. Infinity-Cache "
                            "hits (upper bound on HBM bytes)",
                    "source": os.path.relpath(os.path.join(dst, f"pmc_{tag}.json"), os.path.join(os.path.dirname(tp))),
                    "l2_hit_rate": out.get("l2_hit_rate"),
                    "kernel_steady_state_ns_rocprof": out.get("scan_steady_state_avg_ns")}
        json.dump(tj, open(tp, "w"), indent=1)


if __name__ == "__main__":
    main()
