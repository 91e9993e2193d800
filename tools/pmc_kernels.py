"""Per-kernel SQ / GRBM counters of rocprofv3 --pmc passes (one pass per counter group, tools/pmc_bench.sh).

    python tools/pmc_kernels.py gpurun_out/pmc_b/p1 gpurun_out/pmc_b/p2 ... --top 12 --csv profiles/r03_pmc_kernels.csv

Per kernel (full template name): dispatches, mean duration (from the passes' own timestamps, so it carries the
counter overhead), every counter's per-dispatch mean, and
  mfma_util   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of SIMD-cycles the matrix
              pipes were busy (GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 = the kernel's cycles)
  clock_ghz   GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md 'DVFS give-back'; reads high below ~0.3 ms)
  sq_busy     SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE
  lds_wait    SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (both quad-cycles per wave)
  bank_confl  SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
"""
import argparse
import csv
import os
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def load(dirs):
    val = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> total
    cnt = defaultdict(lambda: defaultdict(int))  # kernel -> counter -> dispatches
    dur = defaultdict(list)  # kernel -> [ns] (one entry per dispatch per pass)
    for d in dirs:
        path = d if d.endswith('.csv') else os.path.join(d, 'run_counter_collection.csv')
        seen = set()
        for r in csv.DictReader(open(path)):
            k = r['Kernel_Name'].split('(')[0]
            c = r['Counter_Name']
            val[k][c] += float(r['Counter_Value'])
            cnt[k][c] += 1
            key = (r['Dispatch_Id'], k)
            if key not in seen:
                seen.add(key)
                dur[k].append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
    return val, cnt, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dirs', nargs='+')
    ap.add_argument('--top', type=int, default=12)
    ap.add_argument('--csv', default=None)
    args = ap.parse_args()
    val, cnt, dur = load(args.dirs)
    counters = sorted({c for k in val for c in val[k]})
    kernels = sorted(dur, key=lambda k: -sum(dur[k]) / max(len(args.dirs), 1))[:args.top]
    rows = []
    for k in kernels:
        per = {c: val[k][c] / cnt[k][c] for c in val[k]}
        mean_ns = sum(dur[k]) / len(dur[k])
        row = {'kernel': k, 'dispatches': max(cnt[k].values()), 'mean_us': mean_ns / 1e3}
        g = per.get('GRBM_GUI_ACTIVE')
        if g:
            row['clock_ghz'] = g / XCDS / mean_ns
            if 'SQ_VALU_MFMA_BUSY_CYCLES' in per:
                row['mfma_util'] = per['SQ_VALU_MFMA_BUSY_CYCLES'] / (SIMDS * g / XCDS)
            if 'SQ_BUSY_CYCLES' in per:
                row['sq_busy'] = per['SQ_BUSY_CYCLES'] / g
        if per.get('SQ_WAVE_CYCLES') and 'SQ_WAIT_INST_LDS' in per:
            row['lds_wait'] = per['SQ_WAIT_INST_LDS'] / per['SQ_WAVE_CYCLES']
        if per.get('SQ_ACTIVE_INST_LDS') and 'SQ_LDS_BANK_CONFLICT' in per:
            row['bank_confl'] = per['SQ_LDS_BANK_CONFLICT'] / per['SQ_ACTIVE_INST_LDS']
        for c in counters:
            if c in per:
                row[c] = per[c]
        rows.append(row)
    derived = ['dispatches', 'mean_us', 'mfma_util', 'clock_ghz', 'sq_busy', 'lds_wait', 'bank_confl']
    for row in rows:
        print(row['kernel'][:100])
        print('   ' + '  '.join(f'{c}={row[c]:.4g}' for c in derived if c in row))
    if args.csv:
        cols = ['kernel'] + derived + counters
        with open(args.csv, 'w', newline='') as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            for row in rows:
                w.writerow({c: (f'{row[c]:.6g}' if isinstance(row.get(c), float) else row.get(c, '')) for c in cols})


if __name__ == '__main__':
    main()
