#!/usr/bin/env python3
"""tests/golden/bench_batch.json: the oracle's answer for the bench headline batch, slice by slice.

Run on a GPU box (the batch comes from the device generator):  python tests/golden/make_bench_golden.py

The headline batch (bench.py defaults: 1024 1080p 4:2:0 High I-slices, QP 22/26/30 groups, seed 0,
BASELINE configs[2]) is generated exactly as bench.make_input makes it; every slice is then cut out
as a standalone Annex-B file (its group's parameter sets + the slice NAL unit; the parallel model
codes each slice from a fresh model, so the slice's output does not depend on the others) and run
through the oracle (tests/_oracle.py slices_p: the CPU restatement of compressor::cabac_decoder,
recode.cpp:1134-1268, with the model reset per slice) on all host threads.  Stored per slice: the
payload size, the CABAC bins the oracle's parse decoded, and the length and SHA-256 of the
oracle's re-coded bytes; plus the input stream's SHA-256 (pins the generator).

bench.py compares the device's per-slice bins and re-coded bytes with this file after its timed
region (so a walker that parses a different bin sequence cannot pass as bit_exact on its own
regeneration verdicts), and tests/test_gpu_parity.py does the same in the GPU suite.
"""
import hashlib
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _slice_job(job):
    path = job
    import _oracle
    data = Path(path).read_bytes()
    _, recs = _oracle.slices_p(data, 0, 1, check_recodable=False)
    (r,) = recs
    return r["status_c"], r["bins"], len(r["recoded"]), hashlib.sha256(r["recoded"]).hexdigest()


def bench_args(slices=1024, seed=0):
    class A:
        pass
    a = A()
    a.mb_width, a.mb_height, a.seed, a.slices = 120, 68, seed, slices
    return a


def oracle_batch(ctx, args, threads=16, progress=print):
    """(stream bytes, per-slice records) for bench.make_input(ctx, args.slices, 0, args)."""
    import multiprocessing as mp

    import bench
    data = bench.make_input(ctx, args.slices, 0, args)
    recs = []
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for j, qp in enumerate(bench.QPS):
            k = (args.slices - j + 2) // 3
            if not k:
                continue
            group = ctx.synthesize(bench.synth_params(qp, args.seed + j, args), k)
            head, nals = bench._split_slices(group)
            assert len(nals) == k
            for i, nal in enumerate(nals):
                p = os.path.join(td, f"g{j}_{i}.264")
                Path(p).write_bytes(head + nal)
                paths.append(p)
        t0 = time.perf_counter()
        with mp.get_context("spawn").Pool(threads) as pool:
            out = pool.map(_slice_job, paths, chunksize=4)
        progress(f"oracle: {len(paths)} slices on {threads} processes in {time.perf_counter() - t0:.1f} s")
    for st, bins, n, h in out:
        recs.append({"status": st, "bins": bins, "recoded_len": n, "recoded_sha256": h})
    return data, recs


def main():
    import avrecode_amd as avr
    args = bench_args()
    with avr.Context(0) as ctx:
        data, recs = oracle_batch(ctx, args)
        ps = avr.parse_stream(data)
    assert len(ps.descs) == len(recs) == args.slices
    g = {
        "config": {"slices": args.slices, "mb": [args.mb_width, args.mb_height], "seed": args.seed,
                   "qp_groups": [22, 26, 30], "model": "parallel (P64)"},
        "stream_sha256": hashlib.sha256(data).hexdigest(),
        "stream_bytes": len(data),
        "bins_total": sum(r["bins"] for r in recs),
        "recoded_total": sum(r["recoded_len"] for r in recs),
        "slices": [{"payload_size": int(ps.descs[k]["payload_size"]), **recs[k]} for k in range(len(recs))],
    }
    assert all(r["status"] == 0 for r in recs)
    out = ROOT / "tests" / "golden" / "bench_batch.json"
    if len(sys.argv) > 1:
        out = Path(sys.argv[1])
    out.write_text(json.dumps(g, separators=(",", ":")) + "\n")
    print(f"wrote {out}: {args.slices} slices, {g['bins_total']} bins, {g['recoded_total']} re-coded bytes")


if __name__ == "__main__":
    main()
