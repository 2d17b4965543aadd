#!/usr/bin/env python
"""Median / min / max per arm of an alternating A/B directory (tools/ab_args.sh): markdown table."""
import glob
import json
import os
import sys

import numpy as np


def main(d):
    arms = {}
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        name = os.path.basename(f).rsplit(".", 2)[0]
        try:
            j = json.load(open(f))
        except Exception:
            continue
        arms.setdefault(name, []).append(j)
    print("| arm | runs | ms/step median | min | max | spread | % verified | % sound |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for name, js in arms.items():
        ms = np.array([j["ms_per_step"] for j in js])
        pv = sorted({j["pct_verified"] for j in js})
        ps = sorted({j["pct_verified_sound"] for j in js})
        print(f"| {name} | {len(ms)} | {np.median(ms):.1f} | {ms.min():.1f} | {ms.max():.1f} | "
              f"{100 * (ms.max() - ms.min()) / np.median(ms):.1f} % | {'/'.join(map(str, pv))} | "
              f"{'/'.join(map(str, ps))} |")


if __name__ == "__main__":
    main(sys.argv[1])
