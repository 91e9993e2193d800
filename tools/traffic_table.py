"""Per-launch HBM traffic of the conv kernels against each launch's algorithmic bytes.

    rocprofv3 --pmc FETCH_SIZE -d <dir>/fetch -o run -- python3 tools/traffic_table.py log --out <dir>/fetch/launches.json
    rocprofv3 --pmc WRITE_SIZE -d <dir>/write -o run -- python3 tools/traffic_table.py log --out <dir>/write/launches.json
    python3 tools/traffic_table.py table <dir> [--csv out.csv]

`log` runs training steps of a config (bench.py's step) and records every scd_conv_igemm / scd_conv_wgrad call in
order with its operand shapes; `table` pairs them with the conv dispatches of each PMC pass (same order; a call that
launches more than one dispatch -- > 2 GiB image chunks -- is refused) and prints, per launch of the last step:
algorithmic bytes (every operand read once, every output written once), FETCH (x2, the gfx950 wide-read
correction of MI355X_MICROARCH.md) and WRITE bytes, and their ratio.  Algorithmic bytes:
  igemm: src (n h_s w_s c) + the output (n h w n_out elements: a ConvT's pixel-shuffled store holds as many) + the
         split weights (planes of the launch's arithmetic x K x n_out x 2 B) [+ y of a fused BatchNorm-backward epilogue]
  wgrad: dY rows (n h w R) + X (n h_s w_s C) [+ y of a rows transform] [+ the dy it stores] + the fp32 slabs written
         (splits x R x taps C)
FETCH counts L2 misses that the Infinity Cache may still serve, so a ratio above 1 is re-read traffic past L2.
The per-launch algorithmic bytes are hip.igemm_alg_bytes / hip.wgrad_alg_bytes, the same functions bench.py sums for
roofline.traffic.algorithmic_bytes_per_step (one definition; round 5's table had counted a ConvT forward's output 4x).
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log_main(a):
    import torch
    from multimodal_siamese_cd_amd import hip, parallel, trainers
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager, networks
    hip.load_library()
    dev = torch.device('cuda:0')
    cfg = experiment_manager.load_cfg(a.config)
    if a.math:
        cfg.MODEL.CONV_MATH = a.math
    batch = a.batch or int(cfg.TRAINER.BATCH_SIZE)
    torch.manual_seed(cfg.SEED)
    net = networks.create_network(cfg).to(dev).train()
    opt = torch.optim.AdamW(net.parameters(), lr=float(cfg.TRAINER.LR), weight_decay=0.01, fused=True)
    b = datasets.synthetic_batch(cfg, batch, dev, torch.Generator(device=dev).manual_seed(7))
    calls = []
    step_no = [0]
    orig_ig, orig_wg = hip.conv_igemm, hip.conv_wgrad

    def igemm(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode=0, **kw):
        # bench.py's definition (hip.igemm_alg_bytes, the launch's own arithmetic)
        arith = hip.igemm_arith(src, out_h, out_w, stride, taps, wpk, n_out, dst, store_mode,
                                src_bound=kw.get('src_bound'))
        alg = hip.igemm_alg_bytes(src, out_h, out_w, taps, n_out, dst, arith,
                                  kw['bn_bwd'][0] if kw.get('bn_bwd') is not None else None)
        extra = []
        if kw.get('in_bn') is not None:
            extra.append('in_bn')
        if kw.get('bn_bwd') is not None:
            extra.append('bn_bwd')
        if kw.get('stat_rec') is not None:
            extra.append('stats')
        calls.append(dict(step=step_no[0], kind='igemm', taps=len(taps[0]), stride=stride,
                          shape=f'{src.n}x{src.h}x{src.w}x{src.c} -> {dst.n}x{out_h}x{out_w}x{n_out}',
                          extra=','.join(extra), alg_bytes=int(alg)))
        return orig_ig(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode, **kw)

    def wgrad(d, slabs):
        r, x = d.rows, d.src
        alg = hip.wgrad_alg_bytes(d, slabs.numel() * slabs.element_size())  # bench.py's definition
        extra = []
        if d.rows_y.data:
            extra.append('rows_bn')
        if d.rows_out.data:  # ABI 8: the formed dy stored for the data grad
            extra.append('rows_out')
        if d.src_scale:
            extra.append('src_bn')
        calls.append(dict(step=step_no[0], kind='wgrad', taps=int(d.ntaps), stride=int(d.stride),
                          shape=f'dY {r.n}x{r.h}x{r.w}x{r.c}, X {x.n}x{x.h}x{x.w}x{x.c}', extra=','.join(extra),
                          alg_bytes=int(alg), slab_bytes=int(slabs.numel() * slabs.element_size())))
        return orig_wg(d, slabs)

    hip.conv_igemm, hip.conv_wgrad = igemm, wgrad
    for s in range(a.steps):
        step_no[0] = s
        opt.zero_grad(set_to_none=True)
        loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, 'w') as f:
        json.dump({'config': a.config, 'batch': batch, 'math': net.module.conv_math, 'steps': a.steps,
                   'calls': calls}, f)


def _is_conv(name):
    n = name.split('(')[0].replace('void ', '').replace('scd::', '').strip()
    return n.startswith(('igemm', 'wgrad_halo', 'wgrad_x3', 'wgrad_f32'))


def _dispatches(path, counter):
    """[(dispatch id, kernel name, value KiB)] of the conv kernels, in dispatch order (summed over the counter's
    per-XCD / per-instance rows)."""
    val = defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter or not _is_conv(r['Kernel_Name']):
            continue
        d = int(r['Dispatch_Id'])
        val[d] += float(r['Counter_Value'])
        name[d] = r['Kernel_Name']
    return [(d, name[d], val[d]) for d in sorted(val)]


def table_main(a):
    rows = {}
    for counter, tag in (('FETCH_SIZE', 'fetch'), ('WRITE_SIZE', 'write')):
        d = os.path.join(a.dir, tag)
        csvp = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith('counter_collection.csv')]
        log = json.load(open(os.path.join(d, 'launches.json')))
        disp = _dispatches(csvp[0], counter)
        calls = log['calls']
        if len(disp) != len(calls):
            sys.exit(f'{tag}: {len(disp)} conv dispatches vs {len(calls)} logged calls (chunked launches?)')
        last = log['steps'] - 1
        for i, (c, (_, kname, v)) in enumerate(zip(calls, disp)):
            if c['step'] != last:
                continue
            ent = rows.setdefault(i, dict(c, kernel=kname.split('(')[0].replace('void ', '').replace('scd::', '')))
            ent[tag] = v * 1024.0 * (2.0 if tag == 'fetch' else 1.0)
        meta = log
    out = sorted(rows.values(), key=lambda r: -(r['fetch'] + r['write'] - r['alg_bytes']))
    tot_alg = sum(r['alg_bytes'] for r in out)
    tot_f = sum(r['fetch'] for r in out)
    tot_w = sum(r['write'] for r in out)
    print(f"{meta['config']} bs={meta['batch']} math={meta['math']}: {len(out)} conv launches per step")
    print(f'algorithmic {tot_alg / 1e9:.2f} GB, FETCH x2 {tot_f / 1e9:.2f} GB, WRITE {tot_w / 1e9:.2f} GB, '
          f'traffic / algorithmic {(tot_f + tot_w) / tot_alg:.2f}')
    for kind in ('igemm', 'wgrad'):
        al = sum(r['alg_bytes'] for r in out if r['kind'] == kind)
        tr = sum(r['fetch'] + r['write'] for r in out if r['kind'] == kind)
        print(f'  {kind}: algorithmic {al / 1e9:.2f} GB, traffic {tr / 1e9:.2f} GB ({tr / al:.2f}x)')
    print(f'{"alg MB":>8} {"fetch MB":>9} {"write MB":>9} {"ratio":>6}  kind  taps shape  [extra]  kernel')
    for r in out:
        print(f"{r['alg_bytes'] / 1e6:8.1f} {r['fetch'] / 1e6:9.1f} {r['write'] / 1e6:9.1f} "
              f"{(r['fetch'] + r['write']) / r['alg_bytes']:6.2f}  {r['kind']} {r['taps']} s{r['stride']} {r['shape']} "
              f"[{r['extra']}]  {r['kernel'][:60]}")
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kind', 'taps', 'stride', 'shape', 'extra', 'kernel', 'alg_bytes', 'fetch_bytes_x2',
                        'write_bytes', 'traffic_over_alg'])
            for r in out:
                w.writerow([r['kind'], r['taps'], r['stride'], r['shape'], r['extra'], r['kernel'], r['alg_bytes'],
                            int(r['fetch']), int(r['write']), round((r['fetch'] + r['write']) / r['alg_bytes'], 3)])


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest='cmd', required=True)
    lg = sub.add_parser('log')
    lg.add_argument('--out', required=True)
    lg.add_argument('--config', default='baseline_siamese')
    lg.add_argument('--batch', type=int, default=None)
    lg.add_argument('--math', default=None)
    lg.add_argument('--steps', type=int, default=2)
    tb = sub.add_parser('table')
    tb.add_argument('dir')
    tb.add_argument('--csv', default=None)
    a = ap.parse_args()
    (log_main if a.cmd == 'log' else table_main)(a)


if __name__ == '__main__':
    main()
