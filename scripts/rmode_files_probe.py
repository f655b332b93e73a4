import sys, json, argparse, time
sys.path.insert(0, '.')
import avrecode_amd as avr, bench
ctx = avr.Context(0)
for n in (1, 64, 256, 512):
    a = argparse.Namespace(rfiles=n, file_reps=2)
    t = time.perf_counter()
    r = bench.rmode_files_section(ctx, a)
    print(n, json.dumps(r), f"{time.perf_counter()-t:.1f}s", flush=True)
