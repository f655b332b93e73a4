"""Estimator lookups of the configs[2] batch that fall through the LDS hash to HBM, and the walker
section cycles (experiment tool; needs a -DAVR_PROFILE -DAVR_PROFILE_EST build via AVR_LIBRARY).

  AVR_LIBRARY=... python3 scripts/est_batch_probe.py .
"""
import ctypes, json, sys, argparse
sys.path.insert(0, sys.argv[1])
import torch
import avrecode_amd as avr, bench
from avrecode_amd.batch import DeviceBatch
L = avr.lib()
buf = (ctypes.c_ulonglong * 64)()
with avr.Context(0) as ctx:
    args = argparse.Namespace(mb_width=120, mb_height=68, seed=0)
    b = DeviceBatch(ctx, avr.parse_stream(bench.make_input(ctx, 1024, 0, args)))
    st = torch.cuda.Stream(0)
    out = {}
    for m in (0, 1, 3, 4):
        L.avr_debug_profile(m, buf)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    with torch.cuda.stream(st):
        b.roundtrip_timed(ev, avr.MODEL_PARALLEL, st)
    torch.cuda.synchronize()
    res = {"compress_s": ev[0].elapsed_time(ev[1]) / 1e3, "decompress_s": ev[2].elapsed_time(ev[3]) / 1e3,
           "verdicts_ok": bool((b.verdicts() == 1).all())}
    for m, name in ((0, "compress"), (1, "decompress")):
        L.avr_debug_profile(m, buf)
        v = list(buf)
        res[name] = {"est_lookups": v[22], "est_hbm": v[23], "walker_bins": v[8], "cycles": v[:8],
                     "waits": v[16:22]}
    print(json.dumps(res))
