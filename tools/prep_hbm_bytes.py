#!/usr/bin/env python3
"""HBM bytes per full-prep node of the light prep (k_prep_cull_lanes + k_prep_pk2<mask-in>), from
the FETCH_SIZE / WRITE_SIZE passes of `bench.py --steps S --warmup W --no-cpu` (separate rocprofv3
--pmc runs, MI355X_MICROARCH.md: FETCH_SIZE doubled on gfx950, WRITE_SIZE as is; both are L2
fabric-side requests, so Infinity-Cache hits are included -- an upper bound on HBM bytes).

    python tools/prep_hbm_bytes.py --fetch gpurun_out/pmc_r1e_fetch --write gpurun_out/pmc_r1e_write \
        --log gpurun_out/pmc_fetch.log --steps 2 --warmup 1 --out profiles/k_prep_hbm_bytes_per_node.json

Every full-prep node (children and cache-build root points) runs k_prep_cull_lanes once and one
k_prep_pk2 instance (the cache-build instance for root points), so bytes per node = the two
kernels' bytes summed over all their dispatches / all full-prep nodes of the profiled run.
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(d, counter):
    path = (glob.glob(os.path.join(d, "*counter_collection.csv")) +  # --output-format csv
            glob.glob(os.path.join(d, "*counter_collection_trace.csv")))[0]  # rocpd2csv of the default db
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k] += float(r["Counter_Value"]) * 1024.0  # KB
        n[k] += 1
    return tot, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--log", required=True, help="bench log of the fetch pass (its 'rank 0 totals' line)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--out", required=True)
    ap.add_argument("--replay", type=int, default=1, help="1 if the profiled bench ran its statistics replay (0: --no-replay)")
    a = ap.parse_args()
    fetch, nf = per_kernel(a.fetch, "FETCH_SIZE")
    write, _ = per_kernel(a.write, "WRITE_SIZE")
    tot = None
    line_json = {}
    for line in open(a.log):
        if line.startswith("rank 0 totals:"):
            tot = json.loads(line.split(":", 1)[1])
        if line.startswith("{"):
            line_json = json.loads(line)
    # totals cover the timed steps; the profile also saw the warmup steps and bench.py's untimed
    # replay of the timed steps (the cull statistic pass, MIS/shade) -- same work per step
    nodes = tot["prep_full_nodes"] * ((1 + a.replay) * a.steps + a.warmup) / a.steps
    kernels = [k for k in fetch if k.startswith("k_prep_cull_lanes") or k.startswith("k_prep_pk2")]
    # FETCH_SIZE x2 only for 16-B-per-lane loads (MI355X_MICROARCH.md): k_prep_pk2's light records are
    # buffer_load_dwordx4; k_prep_cull_lanes reads its table with scalar loads (width uncalibrated, x1)
    mult = {k: (2 if k.startswith("k_prep_pk2") else 1) for k in kernels}
    fb = sum(mult[k] * fetch[k] for k in kernels)
    wb = sum(write.get(k, 0.0) for k in kernels)
    out = {
        "kernel": "k_prep_cull_lanes + k_prep_pk2<mask-in> (one full light prep per node)",
        "hbm_bytes_per_node": round((fb + wb) / nodes, 1),
        "fetch_bytes_per_node": round(fb / nodes, 1),
        "write_bytes_per_node": round(wb / nodes, 1),
        "per_kernel_bytes_per_node": {k: round((mult[k] * fetch[k] + write.get(k, 0.0)) / nodes, 1) for k in kernels},
        "dispatches": {k: nf[k] for k in kernels},
        "full_prep_nodes": int(nodes),
        # the profiled binary (bench.py's line names the library it loaded), so a bench line can tell whether these
        # bytes are its own binary's
        "lib_sha256": line_json.get("lib_sha256"),
        "method": "rocprofv3 --pmc FETCH_SIZE (x2 for k_prep_pk2's 16-B-per-lane record loads, gfx950's 64-B tally of 128-B requests; x1 for the cull's scalar loads) and --pmc WRITE_SIZE in "
                  "separate passes over `bench.py --steps %d --warmup %d --no-cpu`; bytes of both kernels over all "
                  "dispatches / full-prep nodes (timed-step count scaled to the profiled steps: warmup + timed%s); "
                  "tools/prep_hbm_bytes.py"
                  % (a.steps, a.warmup, " + replay" if a.replay else ", --no-replay: only the timed steps' kernel instances"),
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
