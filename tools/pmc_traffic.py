"""Per-step HBM traffic of the MFMA conv kernels from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py gpurun_out/pmc_r1 --steps 3 --out profiles/r01_pmc_traffic.json

Expects <dir>/fetch/run_counter_collection.csv and <dir>/write/run_counter_collection.csv from two separate
passes (MI355X_MICROARCH.md 'HBM': FETCH_SIZE and WRITE_SIZE cannot share a pass; both in KiB).
gfx950 correction: FETCH_SIZE reads exactly half the bytes of wide (16 B/lane) coalesced streaming reads, so
it is doubled; WRITE_SIZE is exact for 16 B/lane stores.  The conv kernels' operand loads are 16 B/lane.
"""
import argparse
import csv
import json
import os
from collections import defaultdict

FAMILIES = {'igemm': 'igemm', 'wgrad_': 'wgrad'}  # substring -> family (igemm_f32/_x3/_halo_x3, wgrad_f32/_x3/_halo_x3)


def load(path, counter):
    out = defaultdict(float)
    n = defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        name = r['Kernel_Name']
        if 'wgrad_finalize' in name or 'wgrad_group_sum' in name:
            continue
        for key, fam in FAMILIES.items():
            if key in name:
                out[fam] += float(r['Counter_Value'])
                n[fam] += 1
                break
    return out, n


def per_kernel(path, counter, out):
    """All kernels of the pass: dispatches, counter total (KiB) and KiB per dispatch, largest first."""
    tot = defaultdict(float)
    n = defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        name = r['Kernel_Name'].split('(')[0]
        tot[name] += float(r['Counter_Value'])
        n[name] += 1
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['kernel', 'dispatches', f'{counter}_KiB_total', 'KiB_per_dispatch'])
        for k in sorted(tot, key=lambda k: -tot[k]):
            w.writerow([k, n[k], f'{tot[k]:.1f}', f'{tot[k] / n[k]:.1f}'])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--steps', type=int, required=True, help='training steps covered by the pass')
    ap.add_argument('--out', default=None)
    ap.add_argument('--math', default='h2', help='conv arithmetic the profiled bench ran (bench.py matches it)')
    ap.add_argument('--summaries', default=None,
                    help='prefix for per-kernel CSVs: <prefix>_pmc_fetch_summary.csv / _pmc_write_summary.csv')
    args = ap.parse_args()
    if args.summaries:
        for counter, tag in (('FETCH_SIZE', 'fetch'), ('WRITE_SIZE', 'write')):
            per_kernel(os.path.join(args.dir, tag, 'run_counter_collection.csv'), counter,
                       f'{args.summaries}_pmc_{tag}_summary.csv')
    fetch, nf = load(os.path.join(args.dir, 'fetch', 'run_counter_collection.csv'), 'FETCH_SIZE')
    write, nw = load(os.path.join(args.dir, 'write', 'run_counter_collection.csv'), 'WRITE_SIZE')
    res = {'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over bench.py, '
                     'FETCH_SIZE x2 (gfx950 wide-read correction), KiB x 1024',
           'steps': args.steps, 'math': args.math, 'per_step_bytes': {}, 'launches_per_step': {}}
    total = 0.0
    for fam in FAMILIES.values():
        b = (2.0 * fetch[fam] + write[fam]) * 1024.0 / args.steps
        res['per_step_bytes'][fam] = b
        res['launches_per_step'][fam] = nf[fam] / args.steps
        total += b
    res['per_step_bytes']['total'] = total
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
