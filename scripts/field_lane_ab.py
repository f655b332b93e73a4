"""The configs[4] corpus's P roundtrip (avr_roundtrip_files) timed in this process, for A/B runs of
the field lane (AVR_FIELD_LANE=0 keeps the field kernel after the progressive one on one stream).

  AVR_FIELD_LANE=0 python scripts/field_lane_ab.py > off.json
"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import avrecode_amd as avr
    from avrecode_amd import workloads
    reps = int(os.environ.get("REPS", "5"))
    with avr.Context(0) as ctx:
        files = workloads.corpus(ctx)
        datas = [d for _, d in files]
        total = sum(map(len, datas))
        ctx.roundtrip_files(datas, avr.MODEL_PARALLEL)   # warm-up
        walls, tc, td = [], [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            outs, times = ctx.roundtrip_files(datas, avr.MODEL_PARALLEL)
            walls.append(time.perf_counter() - t0)
            assert all(isinstance(o, bytes) for o in outs)
            tc.append(times["compress_s"])
            td.append(times["decompress_s"])
        sizes = sum(map(len, ctx.compress_files(datas, avr.MODEL_PARALLEL)))
    print(json.dumps({"field_lane": os.environ.get("AVR_FIELD_LANE", "1"), "bytes": total, "avrc_bytes": sizes,
                      "MB_s": total / statistics.median(walls) / 1e6, "walls": walls, "compress_s": tc,
                      "decompress_s": td}))


if __name__ == "__main__":
    main()
