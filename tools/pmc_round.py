"""HBM traffic per round from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

traffic per round = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB, summed over the
kernels of the round and averaged over rounds.  The factor 2 is the gfx950
FETCH_SIZE correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE = RDREQ x 64 B
counts 128-B requests at 64 B); both raw and corrected reads are recorded.

usage: python tools/pmc_round.py <pmc dir> <workload string> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys

ROUND_KERNELS = ("bin_emit_kernel", "transpose_u16_kernel", "bin_serve_kernel", "bin_apply_kernel",
                 "frontier_summary_kernel", "frontier_scan_kernel", "frontier_commit_kernel",
                 "frontier_rebuild_kernel", "frontier_inject_kernel", "round_snapshot_kernel",
                 "round_random_kernel", "stats_kernel", "round_flood_kernel", "frontier_kernel")


def kname(s):
    return s.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1].split("<")[0].replace("void ", "")


def main():
    d, workload, out = sys.argv[1], sys.argv[2], sys.argv[3]
    tot = collections.Counter()
    per_kernel = collections.defaultdict(collections.Counter)
    launches = collections.Counter()
    for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k not in ROUND_KERNELS:
                continue
            c = r["Counter_Name"]
            v = float(r["Counter_Value"])
            tot[c] += v
            per_kernel[k][c] += v
            if c == "FETCH_SIZE":
                launches[k] += 1
    # one snapshot per round (binned engines); the direct path has one round kernel per round
    rounds = launches.get("round_snapshot_kernel") or launches.get("round_random_kernel") or 1
    fetch = tot["FETCH_SIZE"] * 1024 / rounds
    write = tot["WRITE_SIZE"] * 1024 / rounds
    res = {
        "workload": workload,
        "rounds_profiled": rounds,
        "fetch_bytes_raw_per_round": fetch,
        "fetch_bytes_corrected_per_round": 2 * fetch,
        "write_bytes_per_round": write,
        "hbm_bytes_per_launch": 2 * fetch + write,
        "unit_note": "per round of the whole pipeline; FETCH corrected x2 per MI355X_MICROARCH.md §HBM",
        "per_kernel_MB_per_round": {k: {c: v * 1024 / rounds / 1e6 for c, v in cs.items()} for k, cs in per_kernel.items()},
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel_MB_per_round"}))


if __name__ == "__main__":
    main()
