"""Occupancy / load-balance scan of the slice kernels (diagnostic, not the bench).

For each (slice count, QP set) configuration: generate the batch on the device, run one warm-up and
one timed roundtrip, and print compress / decompress ms, bins per slice (min / mean / max) and the
per-bin time of the longest slice.  Shows whether a batch is bound by its largest slice (QP mix) or
by per-CU sharing (4 slices per CU vs 1).

  python scripts/scan.py [--configs 1024:22,26,30 256:22 ...]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["1024:22,26,30", "1024:22", "256:22", "512:22", "1024:30",
                                                     "2048:22,26,30"])
    ap.add_argument("--mb-width", type=int, default=120)
    ap.add_argument("--mb-height", type=int, default=68)
    args = ap.parse_args()
    import numpy as np
    import torch
    import avrecode_amd as avr
    from avrecode_amd.batch import DeviceBatch

    ctx = avr.Context(0)
    stream = torch.cuda.Stream()
    for cfg in args.configs:
        # n:qps[:slice_type[:mb_width:mb_height]]  (slice_type 0 P, 1 B, 2 I)
        f = cfg.split(":")
        n, qps = int(f[0]), [int(q) for q in f[1].split(",")]
        st = int(f[2]) if len(f) > 2 else 2
        mbw, mbh = (int(f[3]), int(f[4])) if len(f) > 4 else (args.mb_width, args.mb_height)
        parts = []
        for j, qp in enumerate(qps):
            k = (n - j + len(qps) - 1) // len(qps)
            if k:
                parts.append(ctx.synthesize(avr.SynthParams(mb_width=mbw, mb_height=mbh,
                                                            slice_type=st, slice_qp=qp, chroma_format_idc=1,
                                                            transform_8x8_mode=1, seed=j), k))
        data = b"".join(parts)
        ps = avr.parse_stream(data)
        b = DeviceBatch(ctx, ps)
        with torch.cuda.stream(stream):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            b.roundtrip_timed(ev, avr.MODEL_PARALLEL, stream)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            b.roundtrip_timed(ev, avr.MODEL_PARALLEL, stream)
            stream.synchronize()
        ok = bool((b.verdicts() == 1).all())
        res = b.results("c")
        bins = res["bins"].astype(np.float64)
        tc = ev[0].elapsed_time(ev[1])
        td = ev[2].elapsed_time(ev[3])
        S = int(ps.descs["payload_size"].sum())
        line = {"config": cfg, "ok": ok, "S": S, "compress_ms": round(tc, 1), "decompress_ms": round(td, 1),
                "MBps": round(len(data) / (tc + td) / 1e3, 1),
                "bins_min_mean_max": [int(bins.min()), int(bins.mean()), int(bins.max())],
                "ns_per_bin_maxslice": [round(tc * 1e6 / bins.max(), 1), round(td * 1e6 / bins.max(), 1)]}
        print(json.dumps(line), flush=True)
        del b
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
