"""Per-step kernel statistics from a rocprofv3 --kernel-trace database (rocpd SQLite, the default output format).

    python tools/rocpd_stats.py <run_results.db> [--per-step-kernel jaccard_multi_partial] [--csv out.csv]

Steps are counted as the dispatches of a kernel that runs once per training step (default: the OutConv head's
forward), so warmup, timed and probe steps all count and each kernel's ms per step is its total time / steps.
Prints the conv (igemm* / wgrad*) and non-conv totals per step, then the kernels by time."""
import argparse
import csv
import sqlite3
import sys


def load(db: str):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration) from kernels group by name").fetchall()
    return [(n, int(k), float(d) / 1e3) for n, k, d in rows]  # us


def short(name: str) -> str:
    n = name.split('(')[0]
    return n.replace('void ', '').replace('scd::', '').strip()


def is_conv(name: str) -> bool:
    s = short(name)
    return s.startswith(('igemm', 'wgrad_halo', 'wgrad_x3', 'wgrad_f32'))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--per-step-kernel', default='conv1x1_fwd_kernel')
    ap.add_argument('--csv', default=None)
    a = ap.parse_args(argv)
    rows = load(a.db)
    steps = sum(k for n, k, _ in rows if a.per_step_kernel in n)
    if steps == 0:
        sys.exit(f'no dispatch of {a.per_step_kernel!r} in {a.db}')
    rows.sort(key=lambda r: -r[2])
    conv = sum(d for n, _, d in rows if is_conv(n)) / steps / 1e3
    other = sum(d for n, _, d in rows if not is_conv(n)) / steps / 1e3
    print(f'steps (dispatches of {a.per_step_kernel}): {steps}')
    print(f'conv kernels   {conv:8.3f} ms/step')
    print(f'other kernels  {other:8.3f} ms/step')
    print(f'total          {conv + other:8.3f} ms/step ({sum(k for _, k, _ in rows) / steps:.0f} launches/step)')
    print(f'{"ms/step":>8} {"calls/step":>10} {"avg us":>8}  kernel')
    for n, k, d in rows:
        print(f'{d / steps / 1e3:8.3f} {k / steps:10.1f} {d / k:8.1f}  {"*" if is_conv(n) else " "} {short(n)[:110]}')
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kernel', 'conv', 'calls_per_step', 'ms_per_step', 'avg_us', 'calls', 'total_us'])
            for n, k, d in rows:
                w.writerow([short(n), int(is_conv(n)), round(k / steps, 2), round(d / steps / 1e3, 4),
                            round(d / k, 2), k, round(d, 1)])


if __name__ == '__main__':
    main()
