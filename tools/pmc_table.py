"""Per-kernel table of rocprofv3 --pmc passes (host only).

usage: python tools/pmc_table.py <pass_dir> [<pass_dir> ...] [--match sptrsv,spmv]

Each pass directory holds pmc_counter_collection.csv (tools/gpu_steps.sh `pmc=` step).  The
counters of all passes are averaged per kernel instantiation and launch, then reported per wave:
instruction counts, and the split of a wave's lifetime (SQ_WAVE_CYCLES, quad-cycles) into issuing
(SQ_ACTIVE_INST_ANY), parked on a wait count or barrier (SQ_WAIT_ANY) and issue-stalled
(SQ_WAIT_INST_ANY) -- the three are disjoint and sum to SQ_WAVE_CYCLES (MI355X_MICROARCH.md,
rocprofv3 PMC slots).
"""
import collections
import csv
import os
import re
import sys

# sptrsv_pipe_kernel<TPB, RPT, EPT, BWD, ADD, SPLIT, LOC, RES>, sptrsv_upper_kernel<TPB, RPU, EPU, BWD, ADD>
PIPE = re.compile(r"sptrsv_pipe_kernel<(\d+), (\d+), (\d+), (\w+), (\w+), (\d+), (\w+), (\w+)>")
UPPER = re.compile(r"sptrsv_upper_kernel<(\d+), (\d+), (\d+), (\w+), (\w+)>")
CHAIN = re.compile(r"sptrsv_chain_kernel<(\d+), (\d+), (\d+), (\w+)>")


def label(name):
    m = PIPE.search(name)
    if m:
        bwd, add, loc, res = (m.group(i) == "true" for i in (4, 5, 7, 8))
        what = "bwd" + (" +add" if add else "") if bwd else ("fwd fused resid" if res else "fwd")
        return f"round-0 {what} <{m.group(1)},{m.group(2)},{m.group(3)}>"
    m = UPPER.search(name)
    if m:
        bwd, add = m.group(4) == "true", m.group(5) == "true"
        return f"upper {'bwd' if bwd else 'fwd'}{' +add' if add else ''} <{m.group(1)},{m.group(2)},{m.group(3)}>"
    m = CHAIN.search(name)
    if m:
        return f"chain{' +add' if m.group(4) == 'true' else ''} <{m.group(1)},{m.group(2)},{m.group(3)}>"
    return re.sub(r"\(.*", "", name).replace("cpk::", "").replace("(anonymous namespace)::", "")[:48]


def load(dirs, match):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        with open(os.path.join(d, "pmc_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if match and not any(s in r["Kernel_Name"] for s in match):
                    continue
                acc[label(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"_launches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


def main(argv):
    match = ["sptrsv", "spmv"]
    dirs = []
    for a in argv:
        if a.startswith("--match="):
            match = [s for s in a.split("=", 1)[1].split(",") if s]
        else:
            dirs.append(a)
    K = load(dirs, match)
    hdr = (f"{'kernel':34s} {'launch':>6s} {'waves':>6s} {'VALU/w':>8s} {'SALU/w':>8s} {'LDS/w':>7s} "
           f"{'VMRD/w':>7s} {'BR/w':>7s} {'cyc/w':>8s} {'issue':>6s} {'parked':>6s} {'stall':>6s} {'VALU%':>6s}")
    print(hdr)
    print("-" * len(hdr))
    for k in sorted(K):
        c = K[k]
        w = c.get("SQ_WAVES", 0.0) or float("nan")
        wc = c.get("SQ_WAVE_CYCLES", float("nan"))

        def pw(n):
            return c.get(n, float("nan")) / w

        def fr(n):
            return c.get(n, float("nan")) / wc
        print(f"{k:34s} {c['_launches']:6d} {w:6.0f} {pw('SQ_INSTS_VALU'):8.0f} {pw('SQ_INSTS_SALU'):8.0f} "
              f"{pw('SQ_INSTS_LDS'):7.0f} {pw('SQ_INSTS_VMEM_RD'):7.0f} {pw('SQ_INSTS_BRANCH'):7.0f} "
              f"{4 * wc / w:8.0f} {fr('SQ_ACTIVE_INST_ANY'):6.2f} {fr('SQ_WAIT_ANY'):6.2f} {fr('SQ_WAIT_INST_ANY'):6.2f} "
              f"{fr('SQ_ACTIVE_INST_VALU'):6.2f}")
    print("\ncyc/w: cycles per wave (4 x SQ_WAVE_CYCLES / SQ_WAVES); issue / parked / stall: shares of the wave's "
          "lifetime issuing,\nwaiting on a count or barrier, and issue-stalled; VALU%: SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES.")


if __name__ == "__main__":
    main(sys.argv[1:])
