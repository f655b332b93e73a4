"""Estimator-table diagnosis (experiment tool, needs a build with
-DAVR_PROFILE -DAVR_PROFILE_EST: make -C avrecode_amd variant V=est KFLAGS="-DAVR_PROFILE -DAVR_PROFILE_EST",
then AVR_LIBRARY=avrecode_amd/var/est/libavrecode.so): how many SIG/NZ estimator lookups of the
sequential (R-mode) decompress walker fall through the LDS hash table to HBM, per fixture."""
import ctypes
import json
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import avrecode_amd as avr

L = avr.lib()
buf = (ctypes.c_ulonglong * 64)()
out = {}
with avr.Context(0) as ctx:
    for name in ("realshort.mp4", "cockatoo.mp4"):
        data = (ROOT / "tests" / "fixtures" / name).read_bytes()
        c = ctx.compress(data, avr.MODEL_REFERENCE)
        for m in (0, 1, 3, 4):
            L.avr_debug_profile(m, buf)
        t = time.perf_counter()
        back = ctx.decompress(c)
        dt = time.perf_counter() - t
        assert back == data
        L.avr_debug_profile(4, buf)
        v = list(buf)
        out[name] = {"decompress_s": round(dt, 3), "walker_bins": v[8], "est_lookups": v[22], "est_hbm": v[23],
                     "hbm_frac": round(v[23] / max(1, v[22]), 4),
                     "cycles": v[:8], "section_bins": v[8:16],
                     "sub_cycles": v[32:40], "sub_bins": v[40:48]}
print(json.dumps(out, indent=1))
