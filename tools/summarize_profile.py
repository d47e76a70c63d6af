#!/usr/bin/env python3
"""Turn a tools/measure.sh run (gpurun_out/<tag>/) into committed artefacts:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_bench*.json        the bench lines of that pass
  profiles/<tag>_summary.json       top kernels per B=2 forward + per-launch HBM
                                    traffic from the FETCH_SIZE / WRITE_SIZE passes
  profiles/pmc_traffic.json         per-launch traffic that bench.py puts into
                                    roofline.traffic (latest pass)

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read
(MI355X_MICROARCH.md §HBM); every hot kernel here reads 16 B per lane.
Usage: python tools/summarize_profile.py <tag>
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# image-stream kernels (the big image GEMMs run the persistent gemm_w4p_kernel, the fused QKV
# gemm_w4l_kernel, the text stream's gemm_pp)
KEYS = {"attention": "attn_pp_kernel", "mlp_up": "gemm_w4p_kernel<1, false>",
        "gated_gemm": "gemm_w4p_kernel<2, false>", "qkv_gemm": "gemm_w4l_kernel<5, false>"}


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    for f in ("bench", "bench_dit", "bench_int8", "bench_cfg4", "bench_stream2cfg"):
        p = os.path.join(src, f + ".json")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{tag}_{f}.json"))
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    n_attn = sum(int(r["Calls"]) for r in rows if KEYS["attention"] in r["Name"])
    n_fwd = n_attn // 60  # forwards in the traced run (one attention launch per block)
    top = []
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
        setup = r["Name"].startswith("void at::native")  # torch random init / fills, outside the timed loop
        top.append({"kernel": r["Name"][:120], "setup_only": setup, "calls": int(r["Calls"]),
                    "avg_us": float(r["AverageNs"]) / 1e3,
                    "pct": float(r["Percentage"]), "ms_per_forward": float(r["TotalDurationNs"]) / 1e6 / n_fwd})
    traffic = {}
    for kind in ("fetch", "write"):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, f"pmc_{kind}", "run_counter_collection.csv"))):
            for k, pat in KEYS.items():
                if pat in r["Kernel_Name"]:
                    agg[k].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            traffic.setdefault(k, {})[kind + "_size_kb"] = sum(v) / len(v)
    for k, t in traffic.items():
        t["hbm_bytes_per_launch"] = (2 * t.get("fetch_size_kb", 0) + t.get("write_size_kb", 0)) * 1024
    summary = {"tag": tag, "forwards_traced": n_fwd, "top_kernels": top, "traffic_per_launch": traffic,
               "note": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 (gfx950 FETCH_SIZE halving)"}
    json.dump(summary, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1)
    json.dump({"source": f"profiles/{tag}_summary.json", "traffic_per_launch": traffic},
              open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main()
