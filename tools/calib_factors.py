#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration factors for the QT launch's access patterns from a
tools/fetch_calib.hip profile (pmc_summary.py JSON + the program's "known bytes" line).

    python tools/calib_factors.py calib.json known.txt   ->  "FETCH_FACTOR WRITE_FACTOR"

fetch factor = (FETCH_SIZE of k_slots + k_state) / (their known bytes), i.e. the counter's bytes per
true byte for the launch's own read pattern (8 B per lane over 16-lane rows); write factor =
WRITE_SIZE of the 8-B-per-lane store kernel / its known bytes (k_store8 on the 64 MiB buffer)."""
import json
import re
import sys


def main(calib, known):
    d = json.load(open(calib))
    txt = open(known).read()
    kb = {k: float(v) for k, v in re.findall(r"(k_\w+(?:\(buf\))?) (\d+)", txt)}

    def per(name, ctr):
        for k, v in d.items():
            if k != "_meta" and k.split("(")[0].replace("void ", "").strip() == name and ctr in v:
                return v[ctr] * 1024.0
        raise SystemExit(f"{name} / {ctr} missing from {calib}")

    f = (per("k_slots", "FETCH_SIZE") + per("k_state", "FETCH_SIZE")) / (kb["k_slots"] + kb["k_state"])
    # k_store8 runs on the scrub buffer (512 MiB) 4x per rep and on buf (64 MiB) once: the pmc average
    # over its dispatches mixes the two sizes, so use the total: (4 x 512 + 64) MiB per rep
    w = per("k_store8", "WRITE_SIZE") / ((4 * 512 + 64) / 5 * 1048576.0)
    print(f"{f:.4f} {w:.4f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
