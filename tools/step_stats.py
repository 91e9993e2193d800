"""Per-step kernel statistics from a rocprofv3 `--kernel-trace --stats --output-format csv` run.

    python tools/step_stats.py <kernel_stats.csv | kernel_trace.csv> --per-step-kernel pjaccard_partial [--skip 2]
                               [--csv out.csv]

Steps = the calls of a kernel that runs once per training step (the loss's partial pass: pjaccard_partial for the
supervised trainer, jaccard_multi_partial for the dual-task and MMCR trainers).
  * a kernel_trace.csv (preferred): only the steady-state steps count -- the launches between the (skip+1)-th and the
    last call of the per-step kernel, each interval [loss_i, loss_i+1) one step's launches (rotated) -- so one-time
    work (the model's parameter copies, AdamW's first-step state fills, the synthetic batch) is not spread over the
    steps;
  * a kernel_stats.csv: every launch of the run over all per-step-kernel calls (warmup and one-time work included).
Prints conv (igemm* / wgrad*) and non-conv ms per step and every kernel's ms and calls per step; --csv writes the same
table (per-step columns added to rocprofv3's)."""
import argparse
import csv
import sys


def short(name: str) -> str:
    return name.split('(')[0].replace('void ', '').replace('scd::', '').strip()


def is_conv(name: str) -> bool:
    return short(name).startswith(('igemm', 'wgrad_halo', 'wgrad_x3', 'wgrad_f32'))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('stats')
    ap.add_argument('--per-step-kernel', default='pjaccard_partial')
    ap.add_argument('--csv', default=None)
    ap.add_argument('--skip', type=int, default=2, help='kernel trace: leading steps dropped (warmup)')
    a = ap.parse_args(argv)
    with open(a.stats) as f:
        recs = list(csv.DictReader(f))
    if recs and 'Start_Timestamp' in recs[0]:
        launches = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in recs)
        marks = [i for i, r in enumerate(launches) if short(r[2]).startswith(a.per_step_kernel)]
        if len(marks) < a.skip + 2:
            sys.exit(f'{len(marks)} calls of {a.per_step_kernel!r} in {a.stats}: too few steps after --skip {a.skip}')
        steps = len(marks) - 1 - a.skip
        agg = {}
        for s_, e_, n in launches[marks[a.skip]:marks[-1]]:
            k, d = agg.get(n, (0, 0.0))
            agg[n] = (k + 1, d + (e_ - s_))
        rows = [(n, k, d) for n, (k, d) in agg.items()]
        print(f'steady state: the {steps} steps after the first {a.skip} (kernel trace)')
    else:
        rows = [(r['Name'], int(r['Calls']), float(r['TotalDurationNs'])) for r in recs]
        steps = sum(k for n, k, _ in rows if short(n).startswith(a.per_step_kernel))
    if not steps:
        sys.exit(f'no call of {a.per_step_kernel!r} in {a.stats}')
    rows.sort(key=lambda r: -r[2])
    conv = sum(d for n, _, d in rows if is_conv(n)) / steps / 1e6
    other = sum(d for n, _, d in rows if not is_conv(n)) / steps / 1e6
    print(f'steps (calls of {a.per_step_kernel}): {steps}')
    print(f'conv kernels   {conv:8.3f} ms/step')
    print(f'other kernels  {other:8.3f} ms/step  ({100 * other / (conv + other):.1f}% of kernel time)')
    print(f'{"ms/step":>8} {"calls/step":>10} {"avg us":>8}  kernel')
    for n, k, d in rows:
        print(f'{d / steps / 1e6:8.3f} {k / steps:10.2f} {d / k / 1e3:8.1f}  {"*" if is_conv(n) else " "} {short(n)[:110]}')
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kernel', 'conv', 'ms_per_step', 'calls_per_step', 'avg_us', 'calls', 'total_ns', 'steps'])
            for n, k, d in rows:
                w.writerow([n, int(is_conv(n)), round(d / steps / 1e6, 4), round(k / steps, 3), round(d / k / 1e3, 2),
                            k, int(d), steps])


if __name__ == '__main__':
    main()
