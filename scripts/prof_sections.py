"""Walker section cycle breakdown (needs a build with KFLAGS=-DAVR_PROFILE).

  make -C avrecode_amd clean && make -C avrecode_amd -j8 KFLAGS=-DAVR_PROFILE
  python scripts/prof_sections.py [--slices 128]
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

NAMES = ["slice", "mb_syntax", "residual", "map_decode", "nnz_bins", "map_recode", "levels", "mb_bookkeeping"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, default=128)
    args = ap.parse_args()
    import torch
    import avrecode_amd as avr
    from avrecode_amd.batch import DeviceBatch
    import bench

    class A:
        mb_width, mb_height, seed = 120, 68, 0
    ctx = avr.Context(0)
    data = bench.make_input(ctx, args.slices, 0, A)
    ps = avr.parse_stream(data)
    b = DeviceBatch(ctx, ps)
    L = avr.lib()
    buf = (ctypes.c_ulonglong * 64)()
    L.avr_debug_profile(2, buf)   # clear the generator's counters
    out = {}
    for mode, name in ((0, "compress"), (1, "decompress")):
        L.avr_debug_profile(mode, buf)
    b.roundtrip(avr.MODEL_PARALLEL)
    torch.cuda.synchronize()
    assert (b.verdicts() == 1).all()
    for mode, name in ((0, "compress"), (1, "decompress")):
        L.avr_debug_profile(mode, buf)
        v = list(buf)
        bins = v[8] or 1
        out[name] = {"bins": v[8],
                     "cycles": {NAMES[i]: v[i] for i in range(8)},
                     "section_bins": {NAMES[i]: v[8 + i] for i in range(8)},
                     "cycles_per_slice_bin": {NAMES[i]: round(v[i] / bins, 1) for i in range(8)},
                     "cycles_per_section_bin": {NAMES[i]: round(v[i] / max(1, v[8 + i]), 1) for i in range(8)},
                     "waits_per_bin": {"walker_push": round(v[16] / bins, 1), "modeler_take": round(v[17] / bins, 1),
                                       "modeler_push": round(v[18] / bins, 1), "coder_take": round(v[19] / bins, 1),
                                       "modeler_total": round(v[20] / bins, 1), "coder_total": round(v[21] / bins, 1)},
                     "ecache": {"lookups": v[22], "misses": v[23], "nz_lookups": v[24]}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
