"""Where the configs[4] corpus's P-model time goes: each file's slice payload sizes (largest
first) and its P compress / decompress wall time alone, then the whole corpus as one batch.
Run on the GPU box: python3 scripts/long_slice_probe.py > gpurun_out/<tag>/long_slice.json"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import avrecode_amd as avr  # noqa: E402
from avrecode_amd import workloads  # noqa: E402


def main():
    ctx = avr.Context(0)
    files = workloads.corpus(ctx)
    out = {"files": {}}
    only = os.environ.get("PROBE_ONLY")
    for name, data in files:
        if only and only not in name:
            continue
        sizes = sorted(avr.slice_payload_sizes(data).tolist(), reverse=True)
        rec = {"bytes": len(data), "slices": len(sizes), "largest_payloads": sizes[:6]}
        c = ctx.compress(data, avr.MODEL_PARALLEL)
        t0 = time.perf_counter()
        c = ctx.compress(data, avr.MODEL_PARALLEL)
        t1 = time.perf_counter()
        d = ctx.decompress(c)
        t2 = time.perf_counter()
        assert d == data
        rec.update(compress_s=t1 - t0, decompress_s=t2 - t1, ratio=len(c) / len(data))
        info, _ = avr.describe_container(c)
        seams = [len(b["seams"]) // 2 for b in info["blocks"] if "seams" in b]
        rec.update(split_blocks=len(seams), seams_bytes=sum(seams))
        if seams and os.environ.get("PROBE_SAVE"):
            Path(os.environ["PROBE_SAVE"]).mkdir(parents=True, exist_ok=True)
            (Path(os.environ["PROBE_SAVE"]) / f"{name}.264").write_bytes(data)
        out["files"][name] = rec
        print(name, json.dumps(rec), file=sys.stderr, flush=True)
    if only:
        print(json.dumps(out))
        return
    datas = [d for _, d in files]
    ctx.compress_files(datas, avr.MODEL_PARALLEL)
    t0 = time.perf_counter()
    cs = ctx.compress_files(datas, avr.MODEL_PARALLEL)
    t1 = time.perf_counter()
    pc = ctx.last_phase_times()
    ds = ctx.decompress_files(cs)
    t2 = time.perf_counter()
    pd = ctx.last_phase_times()
    out["batch_phases"] = {"compress": pc, "decompress": pd}
    rt, tm = ctx.roundtrip_files(datas, avr.MODEL_PARALLEL)
    t3 = time.perf_counter()
    rt, tm = ctx.roundtrip_files(datas, avr.MODEL_PARALLEL)
    t4 = time.perf_counter()
    out["roundtrip_files"] = {"wall_s": t4 - t3, "MB_s": sum(map(len, datas)) / (t4 - t3) / 1e6, **tm}
    assert all(a == b for a, b in zip(ds, datas))
    out["batch"] = {"compress_s": t1 - t0, "decompress_s": t2 - t1,
                    "MB_s": sum(map(len, datas)) / (t2 - t0) / 1e6}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
