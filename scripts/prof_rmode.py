"""Walker section cycles of the reference-model (sequential) decompress of a whole file (needs the
AVR_PROFILE build: `make -C avrecode_amd prof`, run with AVR_LIBRARY=avrecode_amd/prof/libavrecode.so).

  python scripts/prof_rmode.py tests/fixtures/cockatoo.mp4
"""
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
SUB = ["mb_start", "mb_skip", "mb_type", "intra_modes", "ref_idx", "mvd", "cbp_t8_qp", "eos_publish"]
NAMES = ["slice", "mb_syntax", "residual", "map_decode", "nnz_bins", "map_recode", "levels", "mb_bookkeeping"]


def main():
    import avrecode_amd as avr
    path = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "tests/fixtures/cockatoo.mp4")
    L = avr.lib()
    buf = (ctypes.c_ulonglong * 64)()
    with avr.Context(0) as ctx:
        if path == "clip":   # BASELINE configs[1]: bench.make_clip (1080p, 64 frames, I + 31 P twice)
            sys.path.insert(0, str(ROOT))
            import bench

            class A:
                mb_width, mb_height = 120, 68
            data = bench.make_clip(ctx, A)
        else:
            data = Path(path).read_bytes()
        avrc = ctx.compress(data, avr.MODEL_REFERENCE)
        L.avr_debug_profile(4, buf)
        t0 = time.perf_counter()
        assert ctx.decompress(avrc) == data
        dt = time.perf_counter() - t0
        L.avr_debug_profile(4, buf)
    v = list(buf)
    mbs = v[40]   # sub-section 0 counts macroblocks
    bins = v[8] or 1
    print(json.dumps({"file": path, "decompress_s": dt, "bins": v[8],
                      "cycles_per_bin": {NAMES[i]: round(v[i] / bins, 1) for i in range(8)},
                      "cycles_per_section_bin": {NAMES[i]: round(v[i] / max(1, v[8 + i]), 1) for i in range(8)},
                      "section_bins": {NAMES[i]: v[8 + i] for i in range(8)},
                      "mb_layer_cycles_per_bin": {SUB[i]: round(v[32 + i] / bins, 1) for i in range(8)},
                      "mb_layer_bins": {SUB[i]: v[40 + i] for i in range(8)},
                      "mb_layer_cycles_per_macroblock": {SUB[i]: round(v[32 + i] / max(1, mbs), 1) for i in range(8)},
                      "walker_push_wait_per_bin": round(v[16] / bins, 1),
                      "coder_take_wait_per_bin": round(v[19] / bins, 1), "coder_total_per_bin": round(v[21] / bins, 1)},
                     indent=1))


if __name__ == "__main__":
    main()
