"""A/B of library builds on the configs[2] batch only (experiment tool): for each build, in its own
process, the 1024-slice batch's device compress and decompress (min over reps, HIP events), and
every slice's verdict.  Runs the list twice in interleaved order.

  python scripts/ab_batch.py avrecode_amd/libavrecode.so avrecode_amd/exp/x/libavrecode.so ...
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import torch, argparse
import avrecode_amd as avr, bench
from avrecode_amd.batch import DeviceBatch
with avr.Context(0) as ctx:
    args = argparse.Namespace(mb_width=120, mb_height=68, seed=0)
    b = DeviceBatch(ctx, avr.parse_stream(bench.make_input(ctx, 1024, 0, args)))
    cs, ds = [], []
    st = torch.cuda.Stream(0)
    for _ in range(int(sys.argv[2])):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        with torch.cuda.stream(st):
            b.roundtrip_timed(ev, avr.MODEL_PARALLEL, st)
        torch.cuda.synchronize()
        cs.append(ev[0].elapsed_time(ev[1]) / 1e3); ds.append(ev[2].elapsed_time(ev[3]) / 1e3)
    v = b.verdicts()
    print(json.dumps({"batch_compress_s": min(cs), "batch_decompress_s": min(ds), "all_bit_exact": bool((v == 1).all()),
                      "recoded": hash(b"".join(b.recoded()[:8]))}))
"""


def main():
    libs = sys.argv[1:]
    res = {l: [] for l in libs}
    for rnd in range(2):
        for lib in (libs if rnd == 0 else libs[::-1]):
            env = dict(os.environ, AVR_LIBRARY=str(Path(lib).resolve()))
            p = subprocess.run([sys.executable, "-c", CHILD, str(ROOT), os.environ.get("AB_REPS", "3")], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(lib, p.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            res[lib].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(lib, res[lib][-1], flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
