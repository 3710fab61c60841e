"""GPU idle gaps in a rocprofv3 kernel trace (diagnostic).

    python tools/trace_gaps.py <run_kernel_trace.csv> [--last-ms 3000] [--top 15]

Over the last --last-ms of the trace (the timed steps of bench.py): busy time (union of kernel
intervals), idle time, and the largest gaps with the kernels on either side.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=3000.0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.trace)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    ks.sort()
    t_end = max(e for _, e, _ in ks)
    t0 = t_end - int(a.last_ms * 1e6)
    ks = [k for k in ks if k[0] >= t0]
    busy, gaps, cur_end, prev = 0, [], None, None
    for s, e, n in ks:
        if cur_end is None:
            busy += e - s
            cur_end, prev = e, n
            continue
        if s > cur_end:
            gaps.append((s - cur_end, prev, n))
            busy += e - s
            cur_end, prev = e, n
        elif e > cur_end:
            busy += e - cur_end
            cur_end, prev = e, n
    span = cur_end - ks[0][0]
    idle = sum(g for g, _, _ in gaps)
    print(f"span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.2f} ms "
          f"({100 * idle / span:.2f} %) in {len(gaps)} gaps, {len(ks)} kernels")
    for g, p, n in sorted(gaps, reverse=True)[: a.top]:
        print(f"{g / 1e3:9.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()
