"""Reference-model compress + decompress of one configs[4] corpus file (default: the 4K 4:4:4
IBBP file, the corpus's longest chain), for a rocprofv3 kernel trace of the R-mode passes
(experiment tool):

  rocprofv3 --kernel-trace --stats -d gpurun_out/rk -o run -- python3 scripts/rmode_kernels_probe.py [index]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import avrecode_amd as avr
from avrecode_amd import workloads


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    with avr.Context(0) as ctx:
        name, data = workloads.corpus(ctx, scale=1.0, fixtures=False)[k]
        t0 = time.perf_counter()
        avrc = ctx.compress(data, avr.MODEL_REFERENCE)
        t1 = time.perf_counter()
        assert ctx.decompress(avrc) == data
        t2 = time.perf_counter()
        print(f"{name}: {len(data)} B, R compress {t1 - t0:.3f} s, decompress {t2 - t1:.3f} s", flush=True)


if __name__ == "__main__":
    main()
