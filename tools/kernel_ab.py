"""Per-kernel device time of rocprofv3 --kernel-trace --stats runs side by side (A/B of library
builds on the same box).   python tools/kernel_ab.py NAME=DIR [NAME=DIR ...]   (DIR holds run_kernel_stats.csv)"""
import csv
import os
import re
import sys


def load(d):
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").strip()
        out[n] = out.get(n, 0.0) + float(r["TotalDurationNs"]) / 1e6
    return out


def main():
    runs = [a.split("=", 1) for a in sys.argv[1:]]
    data = [(name, load(d)) for name, d in runs]
    keys = sorted(set().union(*[set(v) for _, v in data]), key=lambda k: -max(v.get(k, 0) for _, v in data))
    print("%-52s" % "kernel (ms, whole run)" + "".join("%11s" % n for n, _ in data))
    for k in keys:
        if max(v.get(k, 0) for _, v in data) < 0.5:
            continue
        print("%-52s" % k[:52] + "".join("%11.1f" % v.get(k, 0) for _, v in data))
    print("%-52s" % "TOTAL" + "".join("%11.1f" % sum(v.values()) for _, v in data))


if __name__ == "__main__":
    main()
