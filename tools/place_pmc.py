"""Which counters separate a fast record-slab placement from a slow one.

Reads rocprofv3 passes (--pmc <group> --kernel-trace) of tools/place_probe4.py: the engine's first
place_tries x 3 dense rounds are its placement trials (one candidate slab per 3 rounds, the first a
warm-up).  Per candidate: the trial round's device time (bin_emit + transpose_u16 + bin_serve +
bin_apply, rounds 2-3 of the candidate, from the kernel trace of the same pass) and each counter,
per round; then, across the candidates of each pass (each pass is its own process, so its own
placements), the Pearson correlation of every counter with the round time.
usage: python tools/place_pmc.py <dir with pass subdirs> [tries] > summary.txt
"""
import collections
import csv
import glob
import math
import os
import sys

DENSE = ("bin_emit_kernel", "bin_emit_huge_kernel", "transpose_u16_kernel", "bin_serve_kernel", "bin_apply_kernel")


def kname(s):
    return s.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1].split("<")[0].replace("void ", "")


def pearson(x, y):
    n = len(x)
    mx, my = sum(x) / n, sum(y) / n
    sx = math.sqrt(sum((a - mx) ** 2 for a in x))
    sy = math.sqrt(sum((b - my) ** 2 for b in y))
    return sum((a - mx) * (b - my) for a, b in zip(x, y)) / (sx * sy) if sx and sy else float("nan")


def one_pass(d, tries):
    tr = [r for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True) for r in csv.DictReader(open(f))]
    pc = [r for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
          for r in csv.DictReader(open(f))]
    if not tr or not pc:
        return None
    dense = sorted((int(r["Start_Timestamp"]), int(r["Dispatch_Id"]), kname(r["Kernel_Name"]),
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in tr if kname(r["Kernel_Name"]) in DENSE)
    per_round = 4
    trial = dense[:tries * 3 * per_round]
    cnt = collections.defaultdict(dict)
    for r in pc:
        cnt[int(r["Dispatch_Id"])][r["Counter_Name"]] = cnt[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    cands = []
    for c in range(tries):
        rows = trial[(3 * c + 1) * per_round:(3 * c + 3) * per_round]
        if len(rows) < 2 * per_round:
            break
        us = sum(x[3] for x in rows) / 2
        ctr = collections.Counter()
        kus = collections.Counter()
        for _, did, k, dur in rows:
            kus[k] += dur / 2
            for n, v in cnt.get(did, {}).items():
                ctr[n] += v / 2
        cands.append((us, dict(kus), dict(ctr)))
    return cands


def main():
    root = sys.argv[1]
    tries = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        cands = one_pass(d, tries)
        if not cands:
            continue
        names = sorted({n for _, _, c in cands for n in c})
        print(f"== {os.path.basename(d)}: {len(cands)} candidates, trial round {min(c[0] for c in cands):.0f}-"
              f"{max(c[0] for c in cands):.0f} us")
        for us, kus, c in sorted(cands, key=lambda x: x[0]):
            ks = " ".join(f"{k.replace('_kernel', '')}={v:.0f}" for k, v in sorted(kus.items()))
            print(f"  {us:8.0f} us  {ks}  " + " ".join(f"{n}={c.get(n, 0):.4g}" for n in names))
        t = [x[0] for x in cands]
        for n in names:
            print(f"  r({n}, round us) = {pearson([x[2].get(n, 0.0) for x in cands], t):+.2f}")
        for k in sorted({k for _, kus, _ in cands for k in kus}):
            print(f"  r({k} us, round us) = {pearson([x[1].get(k, 0.0) for x in cands], t):+.2f}")


if __name__ == "__main__":
    main()
