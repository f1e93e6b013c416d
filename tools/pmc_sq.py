"""Per-kernel PMC counters of the dense-round kernels, averaged per launch, from rocprofv3 --pmc passes.

usage: python tools/pmc_sq.py <pmc dir> [out.json]
Every *_counter_collection.csv under <pmc dir> is read; counters of one kernel name are summed over
its launches and divided by the launch count of that pass (FETCH/TCC/SQ passes each count launches).
Derived: VALU / LDS / wait shares of the wave cycles, TCP accesses and TCC requests per node.
"""
import collections
import csv
import glob
import json
import os
import sys

KEEP = ("bin_emit_kernel", "bin_emit_huge_kernel", "transpose_u16_kernel", "bin_serve_kernel", "bin_apply_kernel",
        "frontier_scan_kernel", "frontier_commit_kernel", "frontier_bs_emit_kernel", "frontier_bs_test_kernel",
        "xd_count_kernel", "xd_emit_kernel", "xd_bin_kernel", "xd_unperm_kernel", "xd_apply_kernel", "sx_scan_kernel")


def kname(s):
    return s.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1].split("<")[0].replace("void ", "")


def main():
    d = sys.argv[1]
    nodes = float(os.environ.get("PMC_NODES", 1 << 24))
    tot = collections.defaultdict(collections.Counter)
    disp = collections.defaultdict(collections.Counter)  # kernel -> counter -> launches seen
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k not in KEEP:
                continue
            c = r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            key = (k, c, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            if key not in seen:
                seen.add(key)
                disp[k][c] += 1
    res = {}
    for k, cs in tot.items():
        a = {c: v / max(disp[k][c], 1) for c, v in cs.items()}
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY",
                      "SQ_ACTIVE_INST_ANY"):
                if c in a:
                    a["share_" + c] = a[c] / wc
        for c in ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum",
                  "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_VALU", "SQ_INSTS_LDS"):
            if c in a:
                a["per_node_" + c] = a[c] / nodes
        if "TCC_HIT_sum" in a and "TCC_MISS_sum" in a:
            a["tcc_hit_rate"] = a["TCC_HIT_sum"] / max(a["TCC_HIT_sum"] + a["TCC_MISS_sum"], 1)
        a["launches"] = max(disp[k].values())
        res[k] = a
    txt = json.dumps(res, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
