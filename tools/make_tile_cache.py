"""Write a synthetic SpaceNet7-style tile cache (the layout utils/datasets.MultimodalCDDataset reads).

    python tools/make_tile_cache.py <root> [--aois 3] [--size 300 290] [--months 4] [--seed 0]

<root>/metadata.json + <root>/<aoi>/{s1,s2,buildings}/<kind>_<aoi>_<year>_<mm>.npy, float32 (H, W, C): s1 2 bands,
s2 4 bands, buildings 1 channel (0/1, growing over time).  The reference's GeoTIFF reader needs rasterio, which
this image lacks; a real cache is the same arrays written with np.save.
"""
import argparse
import json
import os

import numpy as np


def make(root, aois=3, size=(300, 290), months=4, seed=0):
    rng = np.random.default_rng(seed)
    meta = {}
    for a in range(aois):
        aoi = f'L15-{a:04d}E-{a:04d}N_test'
        h, w = size[0] + a, size[1] + 2 * a
        built = rng.random((h, w, 1)) > 0.9
        entries = []
        for m in range(months):
            year, month = 2018 + (m // 12), 1 + m % 12
            built = built | (rng.random((h, w, 1)) > 0.97)
            for kind, arr in (('s1', rng.random((h, w, 2), dtype=np.float32) * 1.2 - 0.1),
                              ('s2', rng.random((h, w, 4), dtype=np.float32)),
                              ('buildings', built.astype(np.float32))):
                os.makedirs(os.path.join(root, aoi, kind), exist_ok=True)
                np.save(os.path.join(root, aoi, kind, f'{kind}_{aoi}_{year}_{month:02d}.npy'), arr)
            entries.append({'year': year, 'month': month, 's1': True, 's2': True, 'buildings': True,
                            'masked': bool(m == 1 and a == 0)})
        meta[aoi] = entries
    with open(os.path.join(root, 'metadata.json'), 'w') as f:
        json.dump(meta, f)
    return sorted(meta)


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('--aois', type=int, default=3)
    ap.add_argument('--size', type=int, nargs=2, default=(300, 290))
    ap.add_argument('--months', type=int, default=4)
    ap.add_argument('--seed', type=int, default=0)
    a = ap.parse_args()
    print(make(a.root, a.aois, tuple(a.size), a.months, a.seed))
