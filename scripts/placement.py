"""Wave placement of the slice kernels (diagnostic; needs the AVR_PROFILE build).

  make -C avrecode_amd prof
  AVR_LIBRARY=$PWD/avrecode_amd/prof/libavrecode.so python scripts/placement.py [--slices 1024] [--qps 22,26,30]

For each slice: the (XCC, SE, SH, CU, SIMD) of its waves (HW_ID / XCC_ID registers) and the walker's
cycles.  Prints how many walkers share a CU / a SIMD, which roles share SIMDs, and the walker's
cycles per bin against the number of other walkers (and other waves) on its SIMD.
"""
import argparse
import collections
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def decode(hw, xcc):
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    return (xcc & 15, se, sh, cu), simd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, default=1024)
    ap.add_argument("--qps", default="22,26,30")
    ap.add_argument("--save", default="", help="prefix: raw per-slice records (+ bins column) to <prefix>_<kernel>.npy")
    args = ap.parse_args()
    import torch
    import avrecode_amd as avr
    from avrecode_amd.batch import DeviceBatch

    ctx = avr.Context(0)
    qps = [int(q) for q in args.qps.split(",")]
    parts = []
    for j, qp in enumerate(qps):
        k = (args.slices - j + len(qps) - 1) // len(qps)
        parts.append(ctx.synthesize(avr.SynthParams(mb_width=120, mb_height=68, slice_type=2, slice_qp=qp,
                                                    chroma_format_idc=1, transform_8x8_mode=1, seed=j), k))
    groups, g0 = [], 0   # (qp, first slice, end) of each contiguous QP group
    for j, qp in enumerate(qps):
        k = (args.slices - j + len(qps) - 1) // len(qps)
        groups.append((qp, g0, g0 + k))
        g0 += k
    ps = avr.parse_stream(b"".join(parts))
    b = DeviceBatch(ctx, ps)
    b.roundtrip(avr.MODEL_PARALLEL)
    torch.cuda.synchronize()
    assert (b.verdicts() == 1).all()
    bins = b.results("c")["bins"].astype(np.float64)
    L = avr.lib()
    n = len(bins)
    out = {}
    for mode, name, nw in ((0, "compress", 3), (1, "decompress", 2)):
        buf = (ctypes.c_uint32 * (8 * n))()
        assert L.avr_debug_placement(mode, buf, n) == 0
        a = np.frombuffer(buf, dtype=np.uint32).reshape(n, 8).astype(np.int64)
        if args.save:
            np.save(f"{args.save}_{name}.npy", np.concatenate([a, bins[:, None].astype(np.int64)], axis=1))
        cyc = (a[:, 5] - a[:, 4]) % (1 << 32)
        rt = (a[:, 7] - a[:, 6]) % (1 << 32)          # 100 MHz ticks
        mhz = cyc / np.maximum(rt, 1) * 100.0
        cus = collections.defaultdict(list)
        simd_roles = collections.defaultdict(list)
        walker_at = []
        for s in range(n):
            cu, sm0 = decode(int(a[s, 0]), int(a[s, 3]))
            cus[cu].append(s)
            walker_at.append((cu, sm0))
            for w in range(nw):
                cu_w, sm = decode(int(a[s, w]), int(a[s, 3]))
                simd_roles[(cu_w, sm)].append(w)
        walkers_per_simd = collections.Counter(walker_at)
        per = []
        for s in range(n):
            k = walker_at[s]
            per.append((walkers_per_simd[k], len(simd_roles[k]), cyc[s] / bins[s]))
        per = np.array(per)
        span = (int(a[:, 7].max()) - int(a[:, 6].min())) % (1 << 32) / 1e5   # ms (same RTC on every XCD)
        res = {"walker_clock_mhz_min_mean_max": [round(float(mhz.min())), round(float(mhz.mean())), round(float(mhz.max()))],
               "walker_ns_per_bin_min_mean_max": [round(float(x), 1) for x in
                                                  ((rt * 10 / bins).min(), (rt * 10 / bins).mean(), (rt * 10 / bins).max())],
               "span_ms": round(span, 1),
               # the batch's tail: each slice's walker lifetime against the launch's span (one
               # walker per slice, all resident at once): busy = sum of lifetimes / (slices x span)
               "walker_ms_min_median_mean_max": [round(float(x) / 1e5, 2) for x in
                                                 (rt.min(), np.median(rt), rt.mean(), rt.max())],
               "walker_busy_fraction": round(float(rt.sum()) / (n * max(span * 1e5, 1.0)), 3),
               "walker_ms_by_qp": {str(q): round(float(rt[g0:g1].mean()) / 1e5, 2) for q, g0, g1 in groups},
               "cus_used": len(cus), "slices_per_cu": dict(collections.Counter(len(v) for v in cus.values())),
               "walkers_per_simd": dict(collections.Counter(walkers_per_simd.values())),
               "roles_per_simd": dict(collections.Counter(tuple(sorted(v)) for v in simd_roles.values()).most_common(8)),
               "same_simd_waves_of_a_slice": int(sum(1 for s in range(n)
                                                      if len({decode(int(a[s, w]), int(a[s, 3]))[1] for w in range(nw)}) < nw)),
               "cycles_per_bin_by_walkers_on_simd": {int(k): round(float(per[per[:, 0] == k, 2].mean()), 1)
                                                     for k in sorted(set(per[:, 0]))},
               "cycles_per_bin_by_waves_on_simd": {int(k): round(float(per[per[:, 1] == k, 2].mean()), 1)
                                                   for k in sorted(set(per[:, 1]))}}
        out[name] = {k: (str(v) if k == "roles_per_simd" else v) for k, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
