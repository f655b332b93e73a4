"""The bench's R-mode many-files leg once (warm-up) and once traced, for a rocprofv3 kernel trace of
its passes (experiment tool):

  rocprofv3 --kernel-trace --stats -d gpurun_out/rf -o run -- python3 scripts/rmode_files_trace.py [n]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import avrecode_amd as avr
from avrecode_amd import workloads


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    with avr.Context(0) as ctx:
        files = workloads.mixed_files(ctx, n=n)
        datas = [d for _, d in files]
        for it in range(2):
            t0 = time.perf_counter()
            outs = ctx.compress_files(datas, avr.MODEL_REFERENCE)
            t1 = time.perf_counter()
            pc = ctx.last_phase_times()
            back = ctx.decompress_files(outs)
            t2 = time.perf_counter()
            pd = ctx.last_phase_times()
            assert back == datas
            print(f"it {it}: compress {t1 - t0:.3f} s {pc}, decompress {t2 - t1:.3f} s {pd}", flush=True)
        order = sorted(range(len(files)), key=lambda i: -len(datas[i]))
        for i in order[:8]:
            ps = avr.parse_stream(datas[i])
            sz = ps.descs["payload_size"]
            print(f"{files[i][0]}: {len(datas[i])} B, {len(sz)} slices, max slice {int(sz.max())} B", flush=True)


if __name__ == "__main__":
    main()
