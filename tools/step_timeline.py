"""Per-step GPU timeline from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

    python tools/step_timeline.py run_kernel_trace.csv --per-step-kernel pjaccard_partial [--skip 2] [--list]

Steps are split at each launch of the per-step kernel (one per training step).  For every step after ``--skip``
it reports the wall time from the step's first kernel start to the next step's, the summed kernel time, the
idle time between kernels (the part of the step no kernel covers), and the largest gaps with the kernels on
either side.  ``--list`` prints the last full step's launches in order (start offset, duration, gap before).
"""
import argparse
import csv
import re
import statistics


def _short(name, n=90):
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--per-step-kernel", required=True)
    ap.add_argument("--skip", type=int, default=2, help="leading steps to drop (warmup)")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--list", action="store_true")
    args = ap.parse_args()

    rows = []
    with open(args.trace, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if args.per_step_kernel in r[2]]
    if len(marks) < args.skip + 2:
        raise SystemExit(f"only {len(marks)} steps in the trace")
    # A step runs from the launch after the previous loss kernel's step boundary: split at the per-step kernel and
    # take each interval [mark_i, mark_{i+1}) as one step (the same kernels, rotated).
    steps = []
    for a, b in zip(marks[args.skip:-1], marks[args.skip + 1:]):
        seg = rows[a:b]
        wall = rows[b][0] - seg[0][0]
        busy = 0
        gaps = []
        end = seg[0][0]
        for i, (s, e, n) in enumerate(seg):
            if s > end:
                gaps.append((s - end, seg[i - 1][2] if i else "", n))
            busy += max(0, e - max(s, end))
            end = max(end, e)
        if rows[b][0] > end:
            gaps.append((rows[b][0] - end, seg[-1][2], rows[b][2]))
        steps.append((wall, busy, gaps, seg))
    us = 1e-3
    walls = [s[0] * us for s in steps]
    busys = [s[1] * us for s in steps]
    idles = [(s[0] - s[1]) * us for s in steps]
    print(f"steps analysed: {len(steps)} (skipped {args.skip})")
    print(f"wall per step    {statistics.median(walls) / 1e3:8.3f} ms (median; min {min(walls) / 1e3:.3f})")
    print(f"kernel-covered   {statistics.median(busys) / 1e3:8.3f} ms")
    print(f"idle between     {statistics.median(idles) / 1e3:8.3f} ms  ({len(steps[-1][2])} gaps in the last step)")
    print(f"launches / step  {len(steps[-1][3])}")
    wall, busy, gaps, seg = steps[-1]
    print(f"\nlargest gaps of the last step (us, kernel before -> kernel after):")
    for g, before, after in sorted(gaps, reverse=True)[:args.top]:
        print(f"  {g * us:8.1f}  {_short(before, 60)}  ->  {_short(after, 60)}")
    hist = {}
    for g, _, _ in gaps:
        k = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else ">=20us"
        hist[k] = hist.get(k, 0) + g * us
    print("idle by gap size (us): " + ", ".join(f"{k} {v:.1f}" for k, v in sorted(hist.items())))
    if args.list:
        t0 = seg[0][0]
        end = t0
        print("\n  offset_us    dur_us   gap_us  kernel")
        for s, e, n in seg:
            print(f"  {(s - t0) * us:9.1f} {(e - s) * us:9.1f} {max(0, s - end) * us:8.1f}  {_short(n)}")
            end = max(end, e)


if __name__ == "__main__":
    main()
