"""One solver iteration from a rocprofv3 --kernel-trace CSV: the kernels between two consecutive
launches of the Krylov product (spmv_stream<EpiKrylov...>), with start offsets, durations and the
gaps between launches (host only).

usage: python tools/iter_trace.py <kernel_trace.csv> [which]   (which: the n-th last iteration, default 2)
"""
import csv
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("cpk::", "").replace("void ", "")
    return n.split("(")[0][:78]


def main(argv):
    rows = list(csv.DictReader(open(argv[0])))
    which = int(argv[1]) if len(argv) > 1 else 2
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "EpiKrylov" in r["Kernel_Name"]]
    if len(idx) < which + 1:
        sys.exit("not enough Krylov products in the trace")
    i0, i1 = idx[-which - 1], idx[-which]
    t0 = int(rows[i0]["Start_Timestamp"])
    prev_end = t0
    busy = 0.0
    print(f"{'start':>8s} {'dur':>7s} {'gap':>6s}  kernel   (us)")
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += (e - s) / 1e3
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(s - prev_end) / 1e3:6.1f}  {short(r['Kernel_Name'])}")
        prev_end = e
    total = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3
    print(f"iteration {total:.1f} us: kernels {busy:.1f}, gaps {total - busy:.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
