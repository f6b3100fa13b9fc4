#!/usr/bin/env python3
"""Turns the rocprofv3 CSVs of a GPU run (gpurun_out/) into the committed summaries (profiles/).

Either rocprofv3's CSV output (--output-format csv) or its default rocpd database converted with
`rocpd2csv -i run_results.db -d DIR` (counters) and `rocpd2summary -i run_results.db -f csv -d DIR`
(kernel stats) is accepted.

    python tools/summarize_profiles.py --tag round1 --stats gpurun_out/prof_r1 \
        --fetch gpurun_out/pmc_r1_fetch --write gpurun_out/pmc_r1_write --sq gpurun_out/pmc_r1_sq \
        --bench gpurun_out/bench_default.log

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) is doubled only for the kernels whose
loads are 16 B per lane (WIDE_LOAD_KERNELS: gfx950 tallies those 128-B requests at 64 B); other
widths are uncalibrated and taken as is (labelled so).  WRITE_SIZE is taken as is; both come from
separate --pmc passes.  They are L2 fabric-side requests, so Infinity-Cache hits are included (an
upper bound on HBM bytes).

VALU: valu_issue_frac = 4 x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs) -- the share of
the SIMDs' issue cycles held by VALU instructions (a wave64 VALU instruction holds its SIMD for at
least 4 cycles, the transcendentals longer: a lower bound, <= 1 up to the GRBM clock estimate).
"""
WIDE_LOAD_KERNELS = ("k_prep_pk2", "k_mis_rays", "k_rays_persistent", "k_extend_brdf", "k_primary")


MIN_US, MAX_CLOCK_GHZ = 100, 2.5  # valu_issue_frac is reported only for dispatches this long and clocks this plausible


def wide(kernel):
    return kernel.startswith(WIDE_LOAD_KERNELS)
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "")


def counters(d):
    # rocprofv3 --output-format csv writes *counter_collection.csv; rocpd2csv (from the default
    # rocpd database output) writes out_counter_collection_trace.csv with the same columns
    path = (glob.glob(os.path.join(d, "*counter_collection.csv")) +
            glob.glob(os.path.join(d, "*counter_collection_trace.csv")))[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: dict(v, dispatches=len(disp[k])) for k, v in agg.items()}


def provenance(lib_path, bench_line=None):
    """what the profiled binary was: the sha256 of the library the GPU run loaded (bench.py prints it in its line;
    else the in-tree file now), the git commit and the tree hash of the library's sources at summarization time
    (the tree hash stays the same across later documentation-only commits)"""
    import hashlib
    import subprocess
    out = {}
    sha = (bench_line or {}).get("lib_sha256")
    if not sha and os.path.exists(lib_path):
        with open(lib_path, "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()
    out["lib_sha256"] = sha

    def git(*a):
        try:
            return subprocess.run(["git", "-C", ROOT] + list(a), capture_output=True, text=True, check=True).stdout.strip()
        except (OSError, subprocess.CalledProcessError):
            return None
    out["head"] = git("rev-parse", "HEAD")
    out["code_tree"] = git("rev-parse", "HEAD:monte_carlo_path_tracing_amd/csrc")
    dirty = git("status", "--porcelain", "--", "monte_carlo_path_tracing_amd/csrc", "include")
    out["code_dirty"] = bool(dirty) if dirty is not None else None
    return out


def pmc_latest(tag, summary):
    """Per-kernel PMC figures bench.py attaches to its roofline objects (profiles/pmc_latest.json):
    valu_issue_frac (module docstring), the effective clock GRBM_GUI_ACTIVE / 8 / duration, and
    HBM-side bytes per dispatch (FETCH_SIZE, x2 for 16-B-per-lane loads, + WRITE_SIZE); the SQ and
    GRBM counters come from separate passes over the same workload, so both are taken per dispatch."""
    ks, sq, hbm = summary.get("kernel_stats", {}), summary.get("sq", {}), summary.get("hbm", {})
    out = {"source": "profiles/%s_summary.json (rocprofv3 --pmc passes; tools/summarize_profiles.py)" % tag,
           "kernels": {}, "provenance": summary.get("provenance")}
    for k, h in hbm.items():
        if not k.startswith("k_") or k not in sq or not h.get("grbm_gui_active"):
            continue
        g = h["grbm_gui_active"] / h["dispatches"]  # summed over the 8 XCDs, per dispatch
        iv = sq[k]["SQ_INSTS_VALU"] / sq[k]["dispatches"]
        e = {"valu_issue_frac": round(4 * iv / (1024 * g / 8), 4),
             "hbm_bytes_per_dispatch": h["fetch_bytes_per_dispatch"] + h["write_bytes_per_dispatch"],
             "fetch_width": "16B/lane (FETCH_SIZE x2)" if wide(k) else "uncalibrated (FETCH_SIZE x1)",
             "dispatches": h["dispatches"]}
        if k in ks:
            e["avg_us"] = ks[k]["avg_us"]
            e["eff_clock_GHz"] = round(g / 8 / (ks[k]["avg_us"] * 1e-6) / 1e9, 3)
            # GRBM_GUI_ACTIVE counts the busy cycles around a dispatch, not its own: for kernels of
            # tens of microseconds it overstates the cycles (an effective clock above the chip's
            # 2.4 GHz), so the issue fraction is not reported there
            if e["avg_us"] < MIN_US or e["eff_clock_GHz"] > MAX_CLOCK_GHZ:
                e["valu_issue_frac"] = None
                e["valu_issue_frac_note"] = ("dropped: %.1f us per dispatch, effective clock %.2f GHz (reported only "
                                             "for >= %d us and <= %.1f GHz)" % (e["avg_us"], e["eff_clock_GHz"], MIN_US,
                                                                                MAX_CLOCK_GHZ))
        out["kernels"][k] = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq")
    ap.add_argument("--bench")
    ap.add_argument("--lib", default=os.path.join(ROOT, "monte_carlo_path_tracing_amd", "libmcpt_hip.so"))
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(a.stats, "*kernel_stats.csv"))
    if stats:
        rows = list(csv.DictReader(open(stats[0])))
    else:  # rocpd2summary -f csv: *_kernels_summary.csv, durations in columns "... (Nsec)"
        rows = [{"Name": r["Name"], "Calls": r["Calls"], "TotalDurationNs": r["Duration (Nsec)"],
                 "AverageNs": r["Average (Nsec)"], "Percentage": r["Percent (Inc)"],
                 "MinNs": r["Min (Nsec)"], "MaxNs": r["Max (Nsec)"]}
                for r in csv.DictReader(open(glob.glob(os.path.join(a.stats, "*kernels_summary.csv"))[0]))]
    with open(os.path.join(out, "%s_kernel_stats.csv" % a.tag), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_us", "percent", "min_us", "max_us"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], "%.3f" % (float(r["TotalDurationNs"]) / 1e6),
                        "%.2f" % (float(r["AverageNs"]) / 1e3), "%.2f" % float(r["Percentage"]),
                        "%.2f" % (float(r["MinNs"]) / 1e3), "%.2f" % (float(r["MaxNs"]) / 1e3)])
    summary = {"kernel_stats": {short(r["Name"]): {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                                   "percent": float(r["Percentage"])} for r in rows}}
    if a.fetch and a.write:
        fc, wc = counters(a.fetch), counters(a.write)
        hbm = {}
        for k in fc:
            if k not in wc:
                continue
            fetch_b = (2 if wide(k) else 1) * fc[k]["FETCH_SIZE"] * 1024
            write_b = wc[k]["WRITE_SIZE"] * 1024
            n = fc[k]["dispatches"]
            hbm[k] = {"dispatches": n, "fetch_bytes_per_dispatch": fetch_b / n,
                      "write_bytes_per_dispatch": write_b / wc[k]["dispatches"],
                      "grbm_gui_active": wc[k].get("GRBM_GUI_ACTIVE")}
        summary["hbm"] = hbm
    if a.sq:
        summary["sq"] = counters(a.sq)
    if a.bench and os.path.exists(a.bench):
        for line in open(a.bench):
            if line.startswith("{"):
                summary["bench"] = json.loads(line)
            if line.startswith("rank 0 totals:"):
                summary["bench_totals"] = json.loads(line.split(":", 1)[1])
    summary["provenance"] = provenance(a.lib, summary.get("bench"))
    with open(os.path.join(out, "%s_summary.json" % a.tag), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    latest = pmc_latest(a.tag, summary)
    if latest["kernels"]:
        # merged into the existing file (one entry per kernel, the newest pass wins), so the summaries of
        # several configurations (C3, C2's k_extend_brdf, ...) can all be present; sources are listed
        path = os.path.join(out, "pmc_latest.json")
        try:
            with open(path) as f:
                old = json.load(f)
        except (OSError, ValueError):
            old = {}
        # one entry per workload (the tag's suffix after the round name: "" = the headline C3, "brdf",
        # "cornell", ...), each kernel naming the summary it came from; bench.py reads its workload's
        # entries.  "kernels" is the headline's, with kernels only other workloads run added
        wl = a.tag.split("_", 1)[1] if "_" in a.tag else "c3"
        configs = dict(old.get("configs", {}))
        prov = latest.get("provenance") or {}
        configs[wl] = {"source": latest["source"], "provenance": prov,
                       "kernels": {k: dict(v, source=latest["source"], lib_sha256=prov.get("lib_sha256"),
                                          head=prov.get("head")) for k, v in latest["kernels"].items()}}
        kernels = {}
        for name in sorted(configs, key=lambda c: c != "c3"):
            for k, v in configs[name]["kernels"].items():
                kernels.setdefault(k, v)
        srcs = sorted({c["source"] for c in configs.values()})
        head_cfg = configs.get("c3", configs[wl])
        latest = {"source": head_cfg["source"], "sources": srcs, "kernels": kernels, "configs": configs,
                  "head": (head_cfg.get("provenance") or {}).get("head"),
                  "code_tree": (head_cfg.get("provenance") or {}).get("code_tree"),
                  "lib_sha256": (head_cfg.get("provenance") or {}).get("lib_sha256")}
        with open(path, "w") as f:
            json.dump(latest, f, indent=1, sort_keys=True)
    print(json.dumps({k: summary[k] for k in summary if k != "sq"}, indent=1)[:3000])


if __name__ == "__main__":
    main()
