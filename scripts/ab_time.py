"""A/B timing of library builds on one GPU (experiment tool): for each build, in its own process,
the reference-model decompress of cockatoo.mp4 (one wavefront walks the file) and the P-mode
decompress of the configs[2] 1024-slice batch, min over reps; outputs must equal the input.

  python scripts/ab_time.py avrecode_amd/libavrecode.so avrecode_amd/var/x/libavrecode.so ...
Runs the list twice in interleaved order (box-to-box and run-to-run drift shows up as spread).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import torch
import avrecode_amd as avr
from avrecode_amd.batch import DeviceBatch
data = open(sys.argv[1] + '/tests/fixtures/cockatoo.mp4', 'rb').read()
out = {}
with avr.Context(0) as ctx:
    cts = []
    for _ in range(int(sys.argv[2])):
        t0 = time.perf_counter(); avrc = ctx.compress(data, avr.MODEL_REFERENCE); cts.append(time.perf_counter() - t0)
    out['rmode_cockatoo_compress_s'] = min(cts)
    ts = []
    for _ in range(int(sys.argv[2])):
        t0 = time.perf_counter(); r = ctx.decompress(avrc); ts.append(time.perf_counter() - t0)
        assert r == data
    out['rmode_cockatoo_decompress_s'] = min(ts)
    if sys.argv[5] == '1':   # the configs[1] clip in the reference model (one wavefront walks it)
        import argparse, bench
        clip = bench.make_clip(ctx, argparse.Namespace(mb_width=120, mb_height=68, seed=0))
        t0 = time.perf_counter(); a = ctx.compress(clip, avr.MODEL_REFERENCE); out['rmode_clip_compress_s'] = time.perf_counter() - t0
        t0 = time.perf_counter(); r = ctx.decompress(a); out['rmode_clip_decompress_s'] = time.perf_counter() - t0
        assert r == clip
    if sys.argv[4] == '1':   # P-mode whole files (latency regime: few slices per CU)
        import argparse, bench
        clip = bench.make_clip(ctx, argparse.Namespace(mb_width=120, mb_height=68, seed=0))
        for name, d in (('cockatoo', data), ('clip', clip)):
            cs, ds = [], []
            for _ in range(3):
                t0 = time.perf_counter(); a = ctx.compress(d, avr.MODEL_PARALLEL); cs.append(time.perf_counter() - t0)
                t0 = time.perf_counter(); r = ctx.decompress(a); ds.append(time.perf_counter() - t0)
                assert r == d
            out['P_' + name + '_compress_s'] = min(cs)
            out['P_' + name + '_decompress_s'] = min(ds)
    if sys.argv[3] == '1':
        import argparse, bench
        args = argparse.Namespace(mb_width=120, mb_height=68, seed=0)
        b = DeviceBatch(ctx, avr.parse_stream(bench.make_input(ctx, 1024, 0, args)))
        cs, ds = [], []
        st = torch.cuda.Stream(0)
        for _ in range(3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            with torch.cuda.stream(st):
                b.roundtrip_timed(ev, avr.MODEL_PARALLEL, st)
            torch.cuda.synchronize()
            cs.append(ev[0].elapsed_time(ev[1]) / 1e3); ds.append(ev[2].elapsed_time(ev[3]) / 1e3)
        assert (b.verdicts() == 1).all()
        out['batch_compress_s'] = min(cs)
        out['batch_decompress_s'] = min(ds)
print(json.dumps(out))
"""


def main():
    libs = sys.argv[1:]
    batch = os.environ.get("AB_BATCH", "1")
    pfiles = os.environ.get("AB_PFILES", "0")
    rclip = os.environ.get("AB_RCLIP", "0")
    reps = os.environ.get("AB_REPS", "2")
    res = {l: [] for l in libs}
    for rnd in range(2):
        for lib in (libs if rnd == 0 else libs[::-1]):
            env = dict(os.environ, AVR_LIBRARY=str(Path(lib).resolve()))
            p = subprocess.run([sys.executable, "-c", CHILD, str(ROOT), reps, batch, pfiles, rclip], env=env, capture_output=True,
                               text=True, timeout=600)
            if p.returncode != 0:
                print(p.stdout, p.stderr[-3000:])
                sys.exit(p.returncode)
            res[lib].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(lib, res[lib][-1], flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
