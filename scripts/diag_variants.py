"""Run the batch roundtrip check under several library builds (experiment tool):
  python scripts/diag_variants.py lib1.so lib2.so ...   (each in its own process, AVR_LIBRARY)"""
import os
import subprocess
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CHILD = r"""
import argparse, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
import avrecode_amd as avr
from avrecode_amd.batch import DeviceBatch
import bench
n = int(sys.argv[2])
with avr.Context(0) as ctx:
    for name in ("realshort.mp4", "cockatoo.mp4"):
        data = open(sys.argv[1] + "/tests/fixtures/" + name, "rb").read()
        print(name, "P roundtrip ok:", ctx.decompress(ctx.compress(data, 1)) == data)
    args = argparse.Namespace(mb_width=120, mb_height=68, seed=0)
    b = DeviceBatch(ctx, avr.parse_stream(bench.make_input(ctx, n, 0, args)))
    b.roundtrip(avr.MODEL_PARALLEL)
    torch.cuda.synchronize()
    v, rd = b.verdicts(), b.results("d")
    bad = np.nonzero(v != 1)[0]
    print("batch", n, "unverified", len(bad), "statuses", sorted(set(rd["status"][bad].tolist())))
"""
for lib in sys.argv[1:]:
    env = dict(os.environ, AVR_LIBRARY=str(Path(lib).resolve()))
    p = subprocess.run([sys.executable, "-c", CHILD, str(ROOT), os.environ.get("N", "12")], env=env,
                       capture_output=True, text=True, timeout=300)
    print("==", lib, "rc", p.returncode)
    print(p.stdout.strip())
    if p.returncode:
        print(p.stderr[-2000:])
        sys.exit(1)
