"""Per-file time and estimator-table fall-through of the configs[4] corpus in the parallel model
(experiment tool).  With the default library: compress_files / decompress_files time of each
corpus file alone.  With AVR_LIBRARY=avrecode_amd/var/est/libavrecode.so (make -C avrecode_amd
variant V=est KFLAGS="-DAVR_PROFILE -DAVR_PROFILE_EST"): also the SIG/NZ estimator lookups of
the parallel kernels and how many of them fell through the LDS hash table to the HBM table.

  python scripts/diag_est_corpus.py [out.json]
"""
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import avrecode_amd as avr
from avrecode_amd import workloads


def main():
    L = avr.lib()
    buf = (ctypes.c_ulonglong * 64)()

    def counters(mode):
        L.avr_debug_profile(mode, buf)
        v = list(buf)
        return {"est_lookups": v[22], "est_hbm": v[23], "hbm_frac": round(v[23] / max(1, v[22]), 4)}

    out = {"library": str(avr.library_path), "files": {}}
    with avr.Context(0) as ctx:
        files = workloads.corpus(ctx, scale=1.0)
        for name, data in files:
            rec = {"bytes": len(data)}
            for m in (0, 1):
                counters(m)
            for tag, model in (("P", avr.MODEL_PARALLEL), ("R", avr.MODEL_REFERENCE)):
                ctx.compress_files([data], model)   # warm-up (buffers)
                for m in (0, 1, 3, 4):
                    L.avr_debug_profile(m, buf)
                t0 = time.perf_counter()
                outs = ctx.compress_files([data], model)
                t1 = time.perf_counter()
                c_comp = counters(0 if tag == "P" else 3)
                c_chk = counters(1)
                back = ctx.decompress_files(outs)
                t2 = time.perf_counter()
                assert back == [data], f"{name} {tag}: not restored"
                c_dec = counters(1 if tag == "P" else 4)
                rec[tag] = {"compress_s": round(t1 - t0, 3), "decompress_s": round(t2 - t1, 3),
                            "compress_est": c_comp, "compress_check_est": c_chk, "decompress_est": c_dec}
            print(name, json.dumps(rec), flush=True)
            out["files"][name] = rec
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
