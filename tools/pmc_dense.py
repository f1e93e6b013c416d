"""HBM traffic of one DENSE round from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of bench.py.

A dense round is one launch each of bin_emit, transpose_u16, bin_serve and bin_apply; bench.py
reports this per-round traffic beside the dense round's algorithmic bytes (roofline.traffic).
traffic = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB: the factor 2 is the gfx950 FETCH_SIZE correction
of MI355X_MICROARCH.md §HBM (FETCH_SIZE = RDREQ x 64 B counts 128-B requests at 64 B).

usage: python tools/pmc_dense.py <pmc dir> <workload string> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys

DENSE = ("bin_emit_kernel", "bin_emit_huge_kernel", "transpose_u16_kernel", "bin_serve_kernel", "bin_apply_kernel")


def kname(s):
    return s.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1].split("<")[0].replace("void ", "")


def main():
    d, workload, out = sys.argv[1], sys.argv[2], sys.argv[3]
    per = collections.defaultdict(collections.Counter)
    launches = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k not in DENSE:
                continue
            c = r["Counter_Name"]
            per[k][c] += float(r["Counter_Value"])
            if c in ("FETCH_SIZE",):
                launches[k] += 1
    rounds = launches["bin_apply_kernel"]
    if not rounds:
        sys.exit("no dense rounds in the counter files")
    kb = {k: {c: v * 1024 / rounds for c, v in cs.items()} for k, cs in per.items()}
    fetch = sum(x.get("FETCH_SIZE", 0) for x in kb.values())
    write = sum(x.get("WRITE_SIZE", 0) for x in kb.values())
    res = {
        "workload": workload,
        "dense_rounds_profiled": rounds,
        "fetch_bytes_raw_per_dense_round": fetch,
        "fetch_bytes_corrected_per_dense_round": 2 * fetch,
        "write_bytes_per_dense_round": write,
        "hbm_bytes_per_dense_round": 2 * fetch + write,
        "unit_note": "per dense round (bin_emit + transpose_u16 + bin_serve + bin_apply); FETCH corrected x2 "
                     "per MI355X_MICROARCH.md §HBM",
        "per_kernel_bytes_per_dense_round": {
            k: {"fetch_corrected": 2 * x.get("FETCH_SIZE", 0), "write": x.get("WRITE_SIZE", 0)} for k, x in kb.items()},
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith("per_kernel")}))


if __name__ == "__main__":
    main()
