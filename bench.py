"""Headline benchmark: input H.264 MB/s (compress + roundtrip), bit-exact, PARALLEL model on the
reference's arithmetic coder (arithmetic_code<uint64_t, uint8_t>, recode.cpp:315-316, 816-820).

Workload (BASELINE.json configs[2]): a synthetic batch of 1024 independent
1080p (120x68 MB) 4:2:0 High-profile CABAC I-slices, QP 22/26/30 by i%3, 8x8 transform on, made by
the device generator (avr_synthesize_stream) before timing.  One step = one roundtrip of the whole
batch, resident in HBM: compress every slice (CABAC decode -> model -> re-encode), derive the
decompress descriptors, decompress every slice (model decode -> CABAC re-encode) and verify the
regenerated payloads + last-byte patch against the input (recode.cpp:1594-1624 per slice).  The
parallel model is the reference model reset per slice and codes its decisions with
the reference's own 64-bit coder; the optional 32-bit P32 coder is measured on the same batch
afterwards and reported as the labelled extra key `p32` (with its container-size delta).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

Weak scaling: every rank roundtrips its own 1024-slice batch (different seeds); slices are
independent in the parallel model, so there is no collective in the timed region.  value = bytes of
input H.264 processed by all ranks / max-over-ranks wall time.

roofline: the dominant slice kernel (compress or decompress, whichever is longer), algorithmic
bytes per launch = S + C (compress reads the S payload bytes and writes C re-coded bytes;
decompress the reverse) over its average launch time from HIP events on the launch stream.
traffic: HBM bytes per launch of that kernel from rocprofv3 FETCH_SIZE/WRITE_SIZE passes
(profiles/<round>_pmc.json, written by scripts/pmc_traffic.py), or null.
cpu_baseline: the oracle (CPU restatement of the reference algorithm, oracle/) compress +
decompress of the first slices of the same batch on one host core (value), and on all host
threads (all_cores), ~10-30 s.
file_roundtrip (rank 0, N=1): the north-star command `recode roundtrip <file>` (recode.cpp:1594-1624)
on whole files from host memory -- both fixtures and the BASELINE configs[1] clip (1080p, 64 frames,
I + 31 P twice, QP 26) -- in both model modes, with the CPU oracle's R-mode single-core roundtrip
beside each, and each call's phase breakdown (demux / upload / kernels / download / container).
corpus: BASELINE configs[4] (N=1: one batch per model; N>1: files dealt to ranks, LPT by bytes).
rmode_files (N=1): the reference model over 256 heterogeneous files at once.
rmode_clips (N=1): the reference model over 512 copies of a real x264 clip, beside the CPU oracle on
every host thread.
stream_shard: BASELINE configs[3] at full length (--stream-leg-seconds, default the config's 600 s of
4K, 18,000 slices, 4.47 GB), one timed step of the sharded container roundtrip, with its own
roofline (and, at N=1, a CPU baseline); at N > 1 the stream is sharded over the ranks (strong
scaling, RCCL gathers and scatter); `--stream-shard` runs it alone.
"""
import argparse
import json
import os
import shutil
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
QPS = (22, 26, 30)
METRIC = "input H.264 MB/s (compress+roundtrip) at 1/2/4/8 GPUs; bit-exact pass"
WORKLOAD = "synthetic batch of independent 1080p CABAC I-slices (BASELINE configs[2])"


def progress(msg):
    """Progress to stderr (long legs must keep writing: the GPU runner treats silence as a hang)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def synth_params(qp, seed, args):
    import avrecode_amd as avr
    return avr.SynthParams(mb_width=args.mb_width, mb_height=args.mb_height, slice_type=2, slice_qp=qp,
                           chroma_format_idc=1, transform_8x8_mode=1, seed=seed)


def make_input(ctx, n, rank, args):
    """Annex-B stream of n slices: three parameter-set groups (QP 22/26/30), i%3 -> QP."""
    parts = []
    for j, qp in enumerate(QPS):
        k = (n - j + 2) // 3
        if k:
            parts.append(ctx.synthesize(synth_params(qp, args.seed + 1000003 * rank + j, args), k))
    return b"".join(parts)


def cpu_threads():
    """Host threads the CPU baseline may use: the process's CPU affinity, capped by the job's
    thread budget (OMP_NUM_THREADS is 16 on the GPU box, a one-GPU share of the node)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def _split_slices(stream):
    """An Annex-B stream's non-slice NAL units (parameter sets, ...) and its slice NAL units
    (nal_unit_type 1 or 5), each with its start code."""
    starts = []
    i = stream.find(b"\x00\x00\x01")
    while i >= 0:
        starts.append(i + 3)
        i = stream.find(b"\x00\x00\x01", i + 3)
    head, nals = b"", []
    for k, a in enumerate(starts):
        b = starts[k + 1] - 3 if k + 1 < len(starts) else len(stream)
        while b > a and stream[b - 1] == 0 and k + 1 < len(starts):
            b -= 1   # a 4-byte start code's leading zero
        unit = b"\x00\x00\x00\x01" + stream[a:b]
        if stream[a] & 0x1F in (1, 5):
            nals.append(unit)
        elif not nals:
            head += unit
    return head, nals


def _cpu_slice_task(job):
    """One slice of the all-cores CPU baseline (a spawned worker process: no GPU state)."""
    path, i = job
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    data = Path(path).read_bytes()
    t0 = time.perf_counter()
    _, recs = _oracle.slices_p(data, i, i + 1, check_recodable=False)
    ok = all(r["status_c"] == 0 and r["status_d"] == 0 for r in recs)
    return ok, time.perf_counter() - t0


def cpu_baseline(ctx, args, n_bytes_hint):
    """The oracle (CPU restatement of the reference) on a bounded sample of the same batch:
    value = the reference's own configuration -- R-mode (one model for the whole file,
    recode.cpp:662-665), one thread (recode.cpp:122) -- `recode_oracle roundtrip` of the first
    slices of the batch written as one Annex-B file; all_cores = the parallel model on every host
    thread, one slice per worker process."""
    import tempfile
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    _oracle.build_oracle()
    t_budget = args.cpu_seconds
    # time one slice per QP group first, then size the sample to the budget
    total_bytes, total_t, slices = 0, 0.0, 0
    k = 1
    while True:
        sample = b"".join(ctx.synthesize(synth_params(qp, args.seed + j, args), k) for j, qp in enumerate(QPS))
        with tempfile.NamedTemporaryFile(suffix=".264", delete=False) as fh:
            fh.write(sample)
        try:
            t0 = time.perf_counter()
            cpu = _oracle_roundtrip_s(fh.name)
            dt = time.perf_counter() - t0
        finally:
            os.unlink(fh.name)
        assert cpu, "oracle R-mode roundtrip failed on the sample"
        total_bytes, total_t, slices = len(sample), sum(cpu), 3 * k
        if dt >= t_budget * 0.5 or k >= 64:
            break
        k = max(k + 1, min(64, int(k * t_budget / max(dt, 1e-3))))
    line = {"value": total_bytes / total_t / 1e6, "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": f"first {slices} slices of the batch ({k} per QP group, {total_bytes} input bytes) as one file, "
                      f"oracle R-mode (reference model) compress+decompress on one thread, {total_t:.1f} s"}
    # all host threads: the same per-slice work, one slice per task, in spawned worker processes
    # (the oracle allocates heavily, so threads in one process do not scale)
    nt = cpu_threads()
    if nt > 1:
        import multiprocessing as mp
        import tempfile
        # sized from the one-thread rate so the pool works ~half the budget (a stable sample, not
        # one slice per worker): bytes = rate x threads x budget / 2, at most 128 slices per QP group
        slice_bytes = total_bytes / max(1, slices)
        want = (total_bytes / total_t) * nt * t_budget / 2
        per = max(-(-2 * nt // 3), min(128, int(want / (3 * slice_bytes)) + 1))
        # one Annex-B file per slice, so a task reads and parses only its own slice
        tmpd = tempfile.mkdtemp(prefix="avr_cpu_")
        paths, nbytes = [], 0
        progress(f"cpu baseline: {3 * per} slices on {nt} host threads")
        for j, qp in enumerate(QPS):
            # one generator launch per QP group (slices in parallel), then cut into standalone
            # streams: the group's parameter sets + one slice NAL unit each
            stream = ctx.synthesize(synth_params(qp, args.seed + j, args), per)
            head, nals = _split_slices(stream)
            for i, nal in enumerate(nals):
                paths.append(os.path.join(tmpd, f"s{j}_{i}.264"))
                Path(paths[-1]).write_bytes(head + nal)
                nbytes += len(nal)
        n = len(paths)
        try:
            with mp.get_context("spawn").Pool(nt) as pool:
                pool.map(_cpu_slice_task, [(paths[0], 0)] * nt)  # warm the workers (imports)
                t0 = time.perf_counter()
                outs = pool.map(_cpu_slice_task, [(q, 0) for q in paths], chunksize=1)
                dt = time.perf_counter() - t0
        finally:
            shutil.rmtree(tmpd, ignore_errors=True)
        assert all(ok for ok, _ in outs)
        line["all_cores"] = {"value": nbytes / dt / 1e6, "unit": "MB/s", "cores": nt,
                             "sample": f"{n} slices ({nbytes} input bytes), parallel model (fresh model per "
                                       f"slice), one slice per task, {nt} worker processes, {dt:.1f} s"}
    return line


CLIP_GOP = 32        # BASELINE configs[1]: 64 frames x 1 slice, GOP I + 31 P (twice), QP 26, 1080p


def make_clip(ctx, args, frames=64):
    """BASELINE configs[1] / SURVEY 8d config 2: a 1080p High 4:2:0 clip, one slice per frame,
    I + 31 P twice, QP 26, seed 0 -- consecutive frames, so the reference model's previous-frame
    nnz contexts (recode.cpp:824-843, 884, 910) are live."""
    import avrecode_amd as avr
    return ctx.synthesize(avr.SynthParams(mb_width=args.mb_width, mb_height=args.mb_height, slice_type=0,
                                          slice_qp=26, chroma_format_idc=1, transform_8x8_mode=1, seed=0,
                                          gop_length=CLIP_GOP), frames)


def _oracle_roundtrip_s(path):
    """CPU oracle, R-mode (the reference's own model and thread count, recode.cpp:122), one core:
    `recode_oracle roundtrip file` -> (compress s, decompress s) as it prints them."""
    import re
    import subprocess
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    _, cli = _oracle.build_oracle()
    r = subprocess.run([str(cli), "roundtrip", str(path)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return None
    m = re.search(r"compress ([0-9.]+)s decompress ([0-9.]+)s", r.stdout)
    return (float(m.group(1)), float(m.group(2))) if m else None


def _round_phases(ph):
    return {k: round(v * 1e3, 3) for k, v in ph.items()} | {"unit": "ms"}


def file_roundtrips(ctx, args):
    """The north-star command, `recode roundtrip <file>` (recode.cpp:1594-1624), on whole files from
    host memory: avr_roundtrip_file = demux + compress (device) + container + decompress (device) +
    byte compare, in the reference model (R), the parallel model (P) and the chained reference model
    (C: R restarted every 16 coded slices).  MB/s = file bytes / wall time of one roundtrip call (median of
    the timed reps after one untimed warm-up; PCIe copies and host container work included).  Beside
    each file: the CPU oracle's R-mode roundtrip on one host core."""
    import tempfile
    import avrecode_amd as avr
    files = [(name, (ROOT / "tests" / "fixtures" / name).read_bytes()) for name in ("realshort.mp4", "cockatoo.mp4")]
    if not args.no_clip:
        files.append(("clip_1080p_64f_IP31_qp26 (configs[1])", make_clip(ctx, args)))
    out = {}
    for name, data in files:
        rec = {"bytes": len(data)}
        for tag, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL), ("C", avr.MODEL_CHAINED)):
            walls, comps, decs, stats = [], [], [], []
            # the first call warms up (buffer allocation); a call of seconds is its own sample
            for it in range(1 + args.file_reps):
                t0 = time.perf_counter()
                avrc, st = ctx.roundtrip(data, model)   # raises on any mismatch
                dt = time.perf_counter() - t0
                if it == 0 and dt < 2.0:
                    continue
                walls.append(dt)
                comps.append(st["compress_s"])
                decs.append(st["decompress_s"])
                stats.append(st)
                if dt >= 2.0:
                    break
            progress(f"file {name} {tag}: {len(data) / walls[0] / 1e6:.2f} MB/s")
            k = sorted(range(len(walls)), key=walls.__getitem__)[len(walls) // 2]
            rec[tag] = {"MB_s": len(data) / walls[k] / 1e6, "wall_s": walls[k], "compress_s": comps[k],
                        "decompress_s": decs[k], "avrc_bytes": len(avrc), "ratio": len(avrc) / len(data),
                        "slices": int(st["slices"]), "coded": int(st["coded_slices"]), "bit_exact": True,
                        "attempts": int(stats[k]["attempts"]),
                        "phases": {"compress": _round_phases(stats[k]["compress_phases"]),
                                   "decompress": _round_phases(stats[k]["decompress_phases"])}}
        if args.no_cpu_baseline:
            out[name] = rec
            continue
        with tempfile.NamedTemporaryFile(suffix=".264", delete=False) as fh:
            fh.write(data)
        try:
            cpu = _oracle_roundtrip_s(fh.name)
        finally:
            os.unlink(fh.name)
        if cpu:
            rec["cpu_oracle_R_1core"] = {"MB_s": len(data) / sum(cpu) / 1e6, "compress_s": cpu[0],
                                         "decompress_s": cpu[1], "cores": 1, "kind": "port"}
        out[name] = rec
    return out


def corpus_section(ctx, args):
    """BASELINE configs[4]: a mixed I/P/B corpus (avrecode_amd/workloads.py: 720p/1080p/4K,
    1/2/4/8/17 slices per frame, IBBP and IP GOPs, 4:2:0/4:2:2/4:4:4, plus the two fixtures) as ONE
    batch through avr_roundtrip_files (batched compress + decompress + byte compare of every file,
    the reference's roundtrip over a corpus; the parallel model's per-slice device check runs only
    for a file whose first container does not come back), in the R, P and chained (C) models.
    MB/s = corpus bytes / (the whole call's wall time, median of reps);
    compression ratio = container bytes / input bytes, P and C against R (the reference model).
    CPU beside it: the oracle's R-mode roundtrip of every file, one core."""
    import tempfile
    import avrecode_amd as avr
    from avrecode_amd import workloads
    files = workloads.corpus(ctx, scale=args.corpus_scale)
    datas = [d for _, d in files]
    total = sum(map(len, datas))
    rec = {"files": len(files), "bytes": total, "names": [n for n, _ in files]}
    sizes = {}
    for tag, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL), ("C", avr.MODEL_CHAINED)):
        walls, tc, td = [], [], []
        for it in range(1 + args.file_reps):
            t0 = time.perf_counter()
            outs, times = ctx.roundtrip_files(datas, model)   # compress, decompress, compare every file
            t2 = time.perf_counter()
            assert all(isinstance(o, bytes) for o in outs), f"corpus {tag}: a file did not come back: {outs}"
            if it == 0 and t2 - t0 < 2.0:
                continue   # warm-up
            walls.append(t2 - t0)
            tc.append(times["compress_s"])
            td.append(times["decompress_s"])
            if t2 - t0 >= 2.0:
                break
        progress(f"corpus {tag}: {total / walls[0] / 1e6:.2f} MB/s")
        k = sorted(range(len(walls)), key=walls.__getitem__)[len(walls) // 2]
        sizes[tag] = [len(o) for o in outs]
        rec[tag] = {"MB_s": total / walls[k] / 1e6, "wall_s": walls[k], "compress_s": tc[k], "decompress_s": td[k],
                    "avrc_bytes": sum(sizes[tag]), "ratio": sum(sizes[tag]) / total, "bit_exact": True}
    rec["ratio_P_over_R"] = rec["P"]["avrc_bytes"] / rec["R"]["avrc_bytes"]
    rec["ratio_C_over_R"] = rec["C"]["avrc_bytes"] / rec["R"]["avrc_bytes"]
    rec["per_file_ratio"] = {n: {"R": sizes["R"][i] / len(d), "P": sizes["P"][i] / len(d), "C": sizes["C"][i] / len(d)}
                             for i, (n, d) in enumerate(files)}
    # the parallel model's long-slice split (avr_set_split_bytes): what it cut, what it costs in bytes
    # (the same corpus compressed without it), per file
    p_outs = ctx.compress_files(datas, avr.MODEL_PARALLEL)
    split0 = ctx.split_bytes
    ctx.split_bytes = 0
    try:
        plain = ctx.compress_files(datas, avr.MODEL_PARALLEL)
    finally:
        ctx.split_bytes = split0
    rec["P_split"] = {"split_bytes": split0, "files": {}}
    for (n, d), o, q in zip(files, p_outs, plain):
        cut = avr.seams_of_container(o)
        if cut:
            rec["P_split"]["files"][n] = {"split_blocks": len(cut), "seams_bytes": sum(x for _, x in cut),
                                          "ratio": len(o) / len(d), "ratio_unsplit": len(q) / len(d)}
    rec["P_split"]["ratio_unsplit"] = sum(map(len, plain)) / total
    if not args.no_cpu_baseline:
        tot = 0.0
        for n, d in files:
            with tempfile.NamedTemporaryFile(suffix=".264", delete=False) as fh:
                fh.write(d)
            try:
                cpu = _oracle_roundtrip_s(fh.name)
            finally:
                os.unlink(fh.name)
            if not cpu:
                tot = None
                break
            tot += sum(cpu)
        if tot:
            rec["cpu_oracle_R_1core"] = {"MB_s": total / tot / 1e6, "wall_s": tot, "cores": 1, "kind": "port"}
    return rec


def rmode_clips_section(ctx, args):
    """The reference model's throughput on a library of short real clips: args.rclips copies of the
    x264 fixture realshort.mp4 (97 KB, 36 slices) as independent files through avr_compress_files /
    avr_decompress_files (the same calls as rmode_files), next to the CPU oracle's R-mode roundtrip
    of the same files on every host thread in the same run.  Each file is one serial chain of the
    reference model (recode.cpp:662-665) on either side; the GPU runs hundreds of chains at once."""
    import avrecode_amd as avr
    clip = (ROOT / "tests" / "fixtures" / "realshort.mp4").read_bytes()
    datas = [clip] * args.rclips
    total = sum(map(len, datas))
    walls, tc, td = [], [], []
    for it in range(1 + args.file_reps):
        t0 = time.perf_counter()
        outs = ctx.compress_files(datas, avr.MODEL_REFERENCE)
        t1 = time.perf_counter()
        back = ctx.decompress_files(outs)
        t2 = time.perf_counter()
        assert back == datas, "R-mode clips: decompress did not restore every file"
        if it == 0:
            continue   # warm-up (buffer allocation)
        walls.append(t2 - t0)
        tc.append(t1 - t0)
        td.append(t2 - t1)
    k = sorted(range(len(walls)), key=walls.__getitem__)[len(walls) // 2]
    progress(f"R-mode clips: {total / walls[k] / 1e6:.2f} MB/s")
    rec = {"files": len(datas), "file": "tests/fixtures/realshort.mp4 (x264, 36 slices)", "bytes": total,
           "model": "reference (R)", "MB_s": total / walls[k] / 1e6, "wall_s": walls[k], "compress_s": tc[k],
           "decompress_s": td[k], "avrc_bytes": sum(map(len, outs)), "bit_exact": True}
    if not args.no_cpu_baseline:
        rec["cpu_baseline"] = rmode_files_cpu(datas)
    return rec


def rmode_files_section(ctx, args):
    """The reference model (R-mode) as throughput: its unit of sequential work is a file
    (DESIGN.md §2), so N independent files go through avr_compress_files / avr_decompress_files at
    once -- every slice of every file in one parallel R-mode compress pass, one workgroup per file
    for the decompress.  The files are a heterogeneous mix (workloads.mixed_files: the configs[4]
    kinds -- 720p/1080p/4K, IBBP/IP, 1-17 slices per frame, 4:2:0/4:2:2/4:4:4, PAFF/MBAFF -- each
    with its own seed and length, and the fixtures), so the per-file load is uneven.  MB/s = bytes /
    (compress + decompress wall time), every file checked byte-exact; phases = where each half's
    wall time went (avr_last_phase_times)."""
    import avrecode_amd as avr
    from avrecode_amd import workloads
    files = workloads.mixed_files(ctx, n=args.rfiles)
    datas = [d for _, d in files]
    total = sum(map(len, datas))
    sizes = sorted(map(len, datas))
    walls, tc, td, phc, phd = [], [], [], [], []
    for it in range(1 + args.file_reps):
        t0 = time.perf_counter()
        outs = ctx.compress_files(datas, avr.MODEL_REFERENCE)
        t1 = time.perf_counter()
        pc = ctx.last_phase_times()
        back = ctx.decompress_files(outs)
        t2 = time.perf_counter()
        pd = ctx.last_phase_times()
        assert back == datas, "R-mode files: decompress did not restore every file"
        if it == 0:
            continue   # warm-up (buffer allocation)
        walls.append(t2 - t0)
        tc.append(t1 - t0)
        td.append(t2 - t1)
        phc.append(pc)
        phd.append(pd)
        if t2 - t0 >= 5.0:
            break
    k = sorted(range(len(walls)), key=walls.__getitem__)[len(walls) // 2]
    progress(f"R-mode files: {total / walls[k] / 1e6:.2f} MB/s")
    rec = {"files": len(files), "kinds": "workloads.mixed_files (configs[4] kinds, per-file seeds and lengths, "
                                         "fixtures every 16th)",
           "bytes": total, "file_bytes_min_median_max": [sizes[0], sizes[len(sizes) // 2], sizes[-1]],
           "model": "reference (R)", "MB_s": total / walls[k] / 1e6, "wall_s": walls[k], "compress_s": tc[k],
           "decompress_s": td[k], "avrc_bytes": sum(map(len, outs)), "bit_exact": True,
           "phases": {"compress": _round_phases(phc[k]), "decompress": _round_phases(phd[k])}}
    if not args.no_cpu_baseline:
        rec["cpu_baseline"] = rmode_files_cpu(datas)
    return rec


def rmode_files_cpu(datas):
    """The same files through the CPU oracle's R-mode roundtrip (`recode_oracle roundtrip`, the
    reference's model on one thread per file, recode.cpp:122), one file per host thread, largest
    first: the all-cores CPU figure beside the GPU's R-mode files throughput."""
    import concurrent.futures as cf
    import subprocess
    import tempfile
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    _, cli = _oracle.build_oracle()
    threads = cpu_threads()
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for i, d in enumerate(datas):
            p = Path(td) / f"f{i}.bin"
            p.write_bytes(d)
            paths.append(p)
        order = sorted(range(len(paths)), key=lambda i: -len(datas[i]))

        def one(i):
            r = subprocess.run([str(cli), "roundtrip", str(paths[i])], capture_output=True, timeout=900)
            return r.returncode == 0

        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(max_workers=threads) as ex:
            ok = all(ex.map(one, order))
        dt = time.perf_counter() - t0
    total = sum(map(len, datas))
    progress(f"R-mode files on {threads} host threads (oracle): {total / dt / 1e6:.2f} MB/s")
    return {"value": total / dt / 1e6, "unit": "MB/s", "cores": threads, "kind": "port", "bit_exact": ok,
            "sample": f"the same {len(datas)} files, oracle R-mode roundtrip (compress + decompress + compare), one "
                      f"file per thread, largest first, {dt:.1f} s"}


def stream_shard_leg(ctx, args, seconds, world, rank, dev, with_cpu):
    """BASELINE configs[3]: ONE 4K stream (1 slice per frame, a 1-s GOP I + 29 P tiled to
    `seconds` with rewritten frame numbers) cut by NAL unit into contiguous slice ranges balanced
    by bytes (shard.partition), one range per GPU.  One timed step is the reference's `roundtrip`
    (recode.cpp:1594-1624) of the whole stream, sharded:
      compress    every rank's device compress of its range, the device pack of its re-coded
                  blocks, the gather to rank 0 (shard.gather_flat over RCCL) and rank 0's Recoded
                  container assembly (avr_assemble_container_into, into one reused buffer);
      decompress  rank 0's plan of that container (decompressor::run's read_packet parse,
                  avr_dec_plan_load: no bytes copied) and the re-coded streams' arena, the scatter of
                  each rank's range of it (shard.scatter_parsed over RCCL), every rank's device
                  decompress + pack, the gather of the regenerated slices to rank 0 and its splice
                  with the container's literals and the last-byte patch (avr_dec_plan_splice).
    The spliced file is compared with the stream outside the timed region.  value = stream bytes /
    max-over-ranks time (strong scaling: the stream is the same at every N).  Returns rank 0's
    record (None elsewhere)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import avrecode_amd as avr
    from avrecode_amd import shard, workloads
    from avrecode_amd.batch import DecompressRange, DeviceBatch

    model = avr.MODEL_PARALLEL
    progress(f"rank {rank}: generating the {seconds}-s stream")
    data = workloads.stream_4k(ctx, seconds=seconds, fps=30, mb_width=args.stream_mb[0], mb_height=args.stream_mb[1])
    progress(f"rank {rank}: {len(data)} bytes; parsing")
    setup = {}
    t = time.perf_counter()
    # rank 0 parses the whole stream (its assembly reads every slice); the other ranks only the
    # payload sizes (the partition) and then their own range
    ps = avr.parse_stream(data) if rank == 0 else None
    sizes = ps.descs["payload_size"] if rank == 0 else avr.slice_payload_sizes(data)
    setup["parse_s"] = time.perf_counter() - t
    progress(f"rank {rank}: parsed {len(sizes)} slices in {setup['parse_s']:.1f} s")
    t = time.perf_counter()
    lo, hi = shard.partition(sizes, world)[rank]
    part = shard.subset(ps, lo, hi) if rank == 0 else avr.parse_stream(data, lo, hi)
    setup["subset_s"] = time.perf_counter() - t
    # what this rank's setup held: slices parsed into descriptors, payload bytes copied (rank 0 the
    # whole stream, the others their own range only)
    setup_work = [len(ps.descs) if rank == 0 else hi - lo,
                  len(ps.arena) if rank == 0 else len(part.arena)]
    t = time.perf_counter()
    batch = DeviceBatch(ctx, part)
    drange = DecompressRange(ctx, dev)
    torch.cuda.synchronize()
    setup["h2d_s"] = time.perf_counter() - t
    progress(f"rank {rank}: slices [{lo}, {hi}) resident on the GPU ({setup['h2d_s']:.1f} s)")
    stream = torch.cuda.Stream(dev)
    mk = lambda: [torch.cuda.Event(enable_timing=True) for _ in range(4)]  # noqa: E731
    gdev = _coll(dev)
    n_mine = hi - lo
    dplan = avr.DecompressPlan() if rank == 0 else None
    # rank 0's host buffers, allocated at the first step and reused: the container and the file
    # (host only) and, page-locked (shard.pinned), the two gathers' destinations and the arena that
    # goes back to the devices -- their copies run as DMA without page faults
    bufs = {}

    def buf(name, need, pin=False):
        b = bufs.get(name)
        if b is None or b.nbytes < need:
            n = need + need // 64 + 4096
            b = bufs[name] = shard.pinned(n) if pin else np.empty(n, dtype=np.uint8)
        return b

    # the compress gather's total: every rank's packed re-coded bytes (at most their payloads' 2x + 256
    # capacity, in practice ~ the stream), sized on the first step
    total_c = len(data) + (1 << 24)

    bins_c = 0   # CABAC bins of this rank's compress (the last step's)

    def step(ev, ph):
        marks = [time.perf_counter()]

        def mark(name):
            marks.append(time.perf_counter())
            ph[name] = ph.get(name, 0.0) + marks[-1] - marks[-2]

        # compress: device compress + pack, results to the host, gather, assembly
        ev[0].record(stream)
        batch.compress(model, stream)
        ev[1].record(stream)
        flat, d_off = batch.pack(stream)
        stream.synchronize()
        mark("compress_s")
        res = batch.results("c")
        nonlocal bins_c
        bins_c = int(res["bins"].sum())
        offs = d_off[:n_mine].cpu().numpy().astype(np.int64)
        ok_c = res["status"] == 0
        lens = np.where(ok_c, res["out_len"], 0).astype(np.int64)
        st = np.where(ok_c, 0, -1).astype(np.int64)
        mark("results_d2h_s")
        g = shard.gather_flat(flat, st, offs, lens, dst=0, device=gdev,
                              out=buf("gather", total_c, pin=True) if rank == 0 else None)
        mark("gather_s")
        avrc = pp = dranges = None
        if g is not None:
            need = avr.container_bound(len(data), len(g[0]), int(np.asarray(g[3], dtype=np.int64).sum()))
            avrc = avr.assemble_container(data, *g, model=model, ps=ps, out=buf("container", need))
        mark("assemble_s")
        # decompress: rank 0 plans the container, every rank regenerates its range
        if rank == 0:
            dplan.load(avrc)
            pp = dplan.parsed(buf("arena", dplan.arena_len, pin=True))
            dranges = shard.partition(pp.descs["payload_size"], world)
        mark("plan_s")
        descs, arena, nd, wl, mw, mh = shard.scatter_parsed(pp, dranges, gdev)
        drange.upload(descs, arena, nd, wl, mw, mh, stream)
        torch.cuda.synchronize()
        mark("scatter_h2d_s")
        ev[2].record(stream)
        drange.run(model, stream)
        ev[3].record(stream)
        dflat, dd_off = drange.pack(stream)
        stream.synchronize()
        mark("decompress_s")
        dres = drange.results()
        dlens = np.where(dres["status"] == 0, dres["out_len"], 0).astype(np.int64)
        doffs = dd_off[:nd].cpu().numpy().astype(np.int64)
        gd = shard.gather_flat(dflat, dres["status"].astype(np.int64), doffs, dlens, dst=0, device=gdev,
                               out=buf("gather_d", len(data) + (1 << 20), pin=True) if rank == 0 else None)
        mark("gather_d_s")
        out = None
        if gd is not None:
            out = dplan.splice(*gd, out=buf("file", len(data)))
        mark("splice_s")
        return avrc, out, int(lens.sum())

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            wph = {}
            step(mk(), wph)
            progress(f"rank {rank}: warm-up step done ({', '.join(f'{k} {v:.1f}' for k, v in wph.items())})")
        evs = [mk() for _ in range(args.stream_steps)]
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        phases = {}
        for k in range(args.stream_steps):
            avrc, out, C = step(evs[k], phases)
            progress(f"rank {rank}: step {k} done")
        torch.cuda.synchronize()
        dist.barrier()
        elapsed = time.perf_counter() - t0
    # the last step's spliced file must be the stream (checked outside the timed region)
    good = True
    if rank == 0:
        good = out is not None and len(out) == len(data) and np.array_equal(out, np.frombuffer(data, dtype=np.uint8))
    mx = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
    bad = torch.tensor([0.0 if good else 1.0], dtype=torch.float64, device=gdev)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(bad, op=dist.ReduceOp.SUM)
    # every rank's setup (times and the work it held), for the record
    mine = torch.tensor([setup["parse_s"], setup["subset_s"], setup["h2d_s"]] + [float(x) for x in setup_work],
                        dtype=torch.float64, device=gdev)
    allsetup = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allsetup, mine)
    t = torch.cat([mx, bad])
    if rank != 0:
        return None
    setup_by_rank = [{"parse_s": round(float(a[0]), 3), "subset_s": round(float(a[1]), 3), "h2d_s": round(float(a[2]), 3),
                      "slices_parsed": int(a[3]), "payload_bytes_copied": int(a[4])} for a in allsetup]
    exact = bool(t[1] == 0)
    t_comp = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs) / 1e3
    t_dec = sum(e[2].elapsed_time(e[3]) for e in evs) / len(evs) / 1e3
    S = int(part.descs["payload_size"].sum())
    dominant, t_dom = ("compress", t_comp) if t_comp >= t_dec else ("decompress", t_dec)
    # the kernel this rank's launches ran (a 4K range of thousands of slices: the persistent queue)
    kernel_name = ctx.slice_kernel(drange.n if dominant == "decompress" else n_mine, part.max_mb_width,
                                   dominant == "decompress")
    rec = {
        "metric": METRIC, "value": len(data) * args.stream_steps / float(t[0]) / 1e6, "unit": "MB/s",
        "n_gpus": world, "steps": args.stream_steps, "warmup": args.warmup,
        "ms_per_step": float(t[0]) / args.stream_steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (device generator, seeded; one GOP tiled)",
        "bit_exact": exact,
        "config": {"workload": "one 4K stream sharded by NAL unit: compress, RCCL gather, container assembly, "
                               "container plan, RCCL scatter, decompress, RCCL gather, splice (BASELINE configs[3])"
                               + ("" if seconds == 600 else f"; REDUCED stream: {seconds} s of the config's 600 s"),
                   "seconds": seconds, "fps": 30, "mb": list(args.stream_mb), "slices": len(ps.descs),
                   "stream_bytes": len(data), "container_bytes": len(avrc), "model": "parallel",
                   "parallelism": f"slice ranges over {world} GPU(s)", "payload_bytes_S_rank0": S,
                   "recoded_bytes_C_rank0": C, "bins_rank0": bins_c, "compress_ms": t_comp * 1e3,
                   "decompress_ms": t_dec * 1e3,
                   "coder": "arithmetic_code<uint64_t,uint8_t>",
                   "setup_s_rank0": {k: round(v, 3) for k, v in setup.items()},
                   "setup_by_rank": setup_by_rank,
                   "step_phases_s_rank0": {k: round(v / args.stream_steps, 3) for k, v in phases.items()}},
        "roofline": {"bound": "hbm", "kernel": kernel_name, "achieved": (S + C) / t_dom / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": (S + C) / t_dom / 1e9 / HBM_PEAK_GBS,
                     "traffic": load_stream_traffic(args, seconds, world, kernel_name),
                     "note": "rank 0's slice range: S + C per launch over the kernel's average HIP-event time"},
        "cpu_baseline": None,
    }
    if with_cpu:
        rec["cpu_baseline"] = stream_cpu_baseline(data, ps, args.cpu_seconds)
    return rec


def stream_cpu_baseline(data, ps, budget_s):
    """The oracle's parallel-model (fresh model per slice) compress + decompress of the stream's
    first GOP, each slice a standalone Annex-B file (the stream's parameter sets + that slice, so a
    call parses only its own slice): on one host core in stream order until ~budget_s of CPU work
    (value), and the whole GOP on all host threads, one slice per worker process (all_cores)."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import tempfile
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    _oracle.build_oracle()
    # the first GOP (30 slices, ~7.4 MB at 4K) lies in the stream's first 32 MB
    n_gop = min(30, len(ps.descs))
    head, nals = _split_slices(bytes(data[:32 << 20]))
    nals = nals[:n_gop]
    done_bytes, t_tot, k = 0, 0.0, 0
    while k < len(nals) and t_tot < budget_s:
        t0 = time.perf_counter()
        _, recs = _oracle.slices_p(head + nals[k], 0, 1, check_recodable=False)
        t_tot += time.perf_counter() - t0
        assert all(r["status_c"] == 0 and r["status_d"] == 0 for r in recs)
        done_bytes += int(ps.descs[k]["payload_size"])
        k += 1
    rec = {"value": done_bytes / t_tot / 1e6, "unit": "MB/s (slice payload bytes)", "cores": 1, "kind": "port",
           "sample": f"first {k} slices of the stream (I + {k - 1} P, {done_bytes} payload bytes), each a standalone "
                     f"file, oracle parallel-model compress + decompress, one thread, {t_tot:.1f} s"}
    threads = cpu_threads()
    with tempfile.TemporaryDirectory() as td:
        jobs = []
        for i, nal in enumerate(nals):
            f = Path(td) / f"s{i}.264"
            f.write_bytes(head + nal)
            jobs.append((str(f), 0))
        t0 = time.perf_counter()
        with cf.ProcessPoolExecutor(max_workers=threads, mp_context=mp.get_context("spawn")) as ex:
            ok = all(r[0] for r in ex.map(_cpu_slice_task, jobs))
        dt = time.perf_counter() - t0
    pay = int(ps.descs["payload_size"][:len(nals)].sum())
    rec["all_cores"] = {"value": pay / dt / 1e6, "unit": "MB/s (slice payload bytes)", "cores": threads,
                        "sample": f"the first GOP ({len(nals)} slices, {pay} payload bytes), one slice per task, "
                                  f"{threads} worker processes, {dt:.1f} s", "ok": ok}
    return rec


_JSON_OUT = sys.stdout


def emit(obj):
    """The bench line: the only text on the process's stdout (see the __main__ block)."""
    print(json.dumps(obj), file=_JSON_OUT, flush=True)


def main_stream_shard(args):
    """`--stream-shard`: configs[3] alone at the full (or --stream-seconds) length, N GPUs."""
    import torch
    import torch.distributed as dist

    import avrecode_amd as avr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = _local_device()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    _init_dist(world, dev)
    ctx = avr.Context(local)
    args.stream_steps = args.steps
    rec = stream_shard_leg(ctx, args, args.stream_seconds, world, rank, dev, with_cpu=False)
    if rank == 0:
        emit(rec)
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


def _backend():
    """The process-group backend: RCCL ("nccl") by default; AVR_DIST_BACKEND=gloo runs the N > 1
    code paths as host collectives (tests: several ranks on one GPU)."""
    return os.environ.get("AVR_DIST_BACKEND", "nccl")


def _local_device():
    """This rank's GPU: LOCAL_RANK, modulo the visible devices (one per rank on a node; the
    multi-process tests put every rank on cuda:0).  device_count does not initialise the GPU."""
    import torch
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return local % max(1, torch.cuda.device_count())


def _coll(dev):
    """Where collective tensors live: the GPU with RCCL, host memory with gloo."""
    import torch
    return dev if _backend() == "nccl" else torch.device("cpu")


def _init_dist(world, dev):
    import datetime

    import torch.distributed as dist
    if dist.is_initialized():
        return
    kw = {"device_id": dev} if _backend() == "nccl" else {}
    if world > 1:
        # a collective that does not complete raises after 5 minutes instead of hanging the run
        # (blocking wait: the caller's wait() sees the timeout), so the configs[3] leg can fail
        # alone without taking the headline line with it
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        dist.init_process_group(_backend(), timeout=datetime.timedelta(seconds=300), **kw)
    else:   # a world-1 RCCL group: the same gather path as N > 1
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group(_backend(), rank=0, world_size=1, **kw)


GOLDEN_BATCH = ROOT / "tests" / "golden" / "bench_batch.json"


def golden_check(batch, data, args):
    """The headline batch against the oracle's answer for it, slice by slice (tests/golden/
    bench_batch.json, tests/golden/make_bench_golden.py: the oracle run on every slice of this
    exact batch): the CABAC bins each slice's parse decoded and the SHA-256 of its re-coded bytes.
    The regeneration verdicts alone do not pin the parse (a walker that parses a different bin
    sequence still round-trips); this does.  None when the batch is not the golden's
    configuration (another seed, size or rank)."""
    import hashlib
    if not GOLDEN_BATCH.exists():
        return None
    g = json.loads(GOLDEN_BATCH.read_text())
    c = g["config"]
    if c["slices"] != args.slices or c["mb"] != [args.mb_width, args.mb_height] or c["seed"] != args.seed:
        return None
    rec = {"golden": str(GOLDEN_BATCH.relative_to(ROOT)), "slices": len(g["slices"])}
    if hashlib.sha256(data).hexdigest() != g["stream_sha256"]:
        return rec | {"match": None, "note": "the generator's stream differs from the golden's: regenerate it"}
    res = batch.results("c")
    recoded = batch.recoded()
    bins_bad = [k for k, s in enumerate(g["slices"]) if int(res["bins"][k]) != s["bins"]]
    sha_bad = [k for k, s in enumerate(g["slices"])
               if len(recoded[k]) != s["recoded_len"] or hashlib.sha256(recoded[k]).hexdigest() != s["recoded_sha256"]]
    return rec | {"bins_total": int(res["bins"].sum()), "bins_total_oracle": g["bins_total"],
                  "recoded_total": sum(map(len, recoded)), "recoded_total_oracle": g["recoded_total"],
                  "slices_bins_differ": len(bins_bad), "slices_recoded_differ": len(sha_bad),
                  "match": not bins_bad and not sha_bad}


def load_traffic(args, kernel):
    """HBM bytes per launch of `kernel` from profiles/<round>_pmc.json (scripts/pmc_traffic.py),
    only when that profile was taken on this batch shape AND on this build of the native sources
    (its source_sha equals avrecode_amd.source_sha() of the tree being measured); else None."""
    import avrecode_amd as avr
    p = ROOT / "profiles" / f"{args.round}_pmc.json"
    if not p.exists():
        return None
    try:
        j = json.loads(p.read_text())
        if j.get("leg", "headline") != "headline" or j.get("slices") != args.slices or \
                j.get("mb") != [args.mb_width, args.mb_height]:
            return None
        if j.get("source_sha") != avr.source_sha():
            progress(f"traffic: {p.name} is from another build of the sources; reporting null")
            return None
        return j["kernels"][kernel]["hbm_bytes_per_launch"]
    except Exception:
        return None


def load_stream_traffic(args, seconds, world, kernel):
    """configs[3]'s kernel: HBM bytes per launch from profiles/<round>_stream_pmc.json
    (scripts/pmc_traffic.py --leg stream_shard, passes over `bench.py --stream-shard` at N = 1), when
    that profile is of this stream and this build of the sources and the leg runs on one GPU (at
    N > 1 each rank's launch covers a different range); else None."""
    import avrecode_amd as avr
    p = ROOT / "profiles" / f"{args.round}_stream_pmc.json"
    if world != 1 or not p.exists():
        return None
    try:
        j = json.loads(p.read_text())
        if j.get("leg") != "stream_shard" or j.get("seconds") != seconds or j.get("mb") != list(args.stream_mb):
            return None
        if j.get("source_sha") != avr.source_sha():
            progress(f"traffic: {p.name} is from another build of the sources; reporting null")
            return None
        return j["kernels"][kernel]["hbm_bytes_per_launch"]
    except Exception:
        return None


def p32_extra(batch, args, stream, mk, n_bytes, C64):
    """The optional P32 container coder (avrecode-amd:P32: the parallel model's decisions through a
    32-bit range coder, avr_engine.h PEncoder / PDecoder -- NOT the reference's arithmetic) on the
    headline batch: the same timed roundtrip steps, bit-exactness, and the container-size delta
    against the u64 coder.  A labelled extra key; the headline value is the u64 coder's."""
    import torch
    import avrecode_amd as avr
    with torch.cuda.stream(stream):
        batch.roundtrip_timed(mk(), avr.MODEL_PARALLEL32, stream)   # warm-up
        stream.synchronize()
        evs = [mk() for _ in range(args.steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            batch.roundtrip_timed(evs[k], avr.MODEL_PARALLEL32, stream)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    v = batch.verdicts()
    C = int(batch.results("c")["out_len"][v == 1].sum())
    # leave the batch's outputs as the headline's (later legs read nothing from it, but be tidy)
    with torch.cuda.stream(stream):
        batch.roundtrip_timed(mk(), avr.MODEL_PARALLEL, stream)
        stream.synchronize()
    return {"coder": "P32 (avrecode-amd:P32; 32-bit range coder, truncated quotient; not the reference's arithmetic)",
            "value": n_bytes * args.steps / elapsed / 1e6, "unit": "MB/s", "ms_per_step": elapsed / args.steps * 1e3,
            "compress_ms": sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps,
            "decompress_ms": sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps,
            "bit_exact": bool((v == 1).all()), "recoded_bytes_C": C,
            "container_delta_vs_u64": C / max(1, C64) - 1.0}


def corpus_sharded(ctx, args, world, rank, dev):
    """BASELINE configs[4] on N GPUs.  R and P: the corpus's files dealt whole to the ranks
    (shard.deal_files, LPT by bytes), each rank's files run as one batch per model
    (avr_roundtrip_files: compress, decompress and byte compare, as the N = 1 corpus leg), no
    collective in the timed region; the reference model runs here as replicas over files (its only
    split).  C: every file's chains split over all ranks (the chained model's
    within-file split: chain ranges on each GPU, RCCL gathers, rank 0 assembles and splices).  MB/s =
    corpus bytes / max-over-ranks wall time."""
    import torch
    import torch.distributed as dist

    import avrecode_amd as avr
    from avrecode_amd import shard, workloads
    files = workloads.corpus(ctx, scale=args.corpus_scale)
    total = sum(len(d) for _, d in files)
    mine = shard.deal_files([len(d) for _, d in files], world)[rank]
    datas = [files[i][1] for i in mine]
    rec = {"files": len(files), "bytes": total, "n_gpus": world, "scaling": "strong",
           "files_rank0": [files[i][0] for i in shard.deal_files([len(d) for _, d in files], world)[0]],
           "C_split": "every file's chains over all ranks (shard.sharded_compress_chained / _decompress_chained)"}
    gdev = _coll(dev)

    def chained_roundtrip():
        # the chained model within each file: every rank runs its range of the file's chains, rank 0
        # assembles the container and splices the file back (compared with the input there)
        good = True
        for _, d in files:
            avrc = shard.sharded_compress_chained(ctx, d, device=gdev)
            if rank == 0:
                avrc = bytes(avrc)
            obj = [avrc]
            dist.broadcast_object_list(obj, src=0)   # the container every rank decompresses
            out = shard.sharded_decompress_chained(ctx, obj[0], device=gdev)
            if rank == 0:
                good = good and out == d
        return good

    for tag, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL), ("C", avr.MODEL_CHAINED)):
        for it in range(2):   # one warm-up pass, one timed
            dist.barrier()
            t0 = time.perf_counter()
            ok = True
            if model == avr.MODEL_CHAINED:
                ok = chained_roundtrip()
            elif datas:
                outs, _ = ctx.roundtrip_files(datas, model)   # compress, decompress, compare
                ok = all(isinstance(o, bytes) for o in outs)
            dt = time.perf_counter() - t0
            mx = torch.tensor([dt], dtype=torch.float64, device=_coll(dev))
            bad = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=_coll(dev))
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(bad, op=dist.ReduceOp.SUM)
            t = torch.cat([mx, bad])
        rec[tag] = {"MB_s": total / float(t[0]) / 1e6, "wall_s": float(t[0]), "bit_exact": bool(t[1] == 0)}
        progress(f"corpus {tag} over {world} GPU(s): {rec[tag]['MB_s']:.2f} MB/s")
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--slices", type=int, default=1024)
    ap.add_argument("--mb-width", type=int, default=120)
    ap.add_argument("--mb-height", type=int, default=68)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--round", default="r06")
    ap.add_argument("--file-reps", type=int, default=3, help="timed reps of a whole-file call under 2 s")
    ap.add_argument("--no-files", action="store_true", help="skip the whole-file roundtrips")
    ap.add_argument("--no-clip", action="store_true", help="skip the configs[1] clip in the file roundtrips")
    ap.add_argument("--no-corpus", action="store_true", help="skip the configs[4] corpus")
    ap.add_argument("--corpus-scale", type=float, default=1.0)
    ap.add_argument("--rfiles", type=int, default=256, help="files in the R-mode many-files leg (0: skip)")
    ap.add_argument("--rclips", type=int, default=512, help="copies of realshort.mp4 in the R-mode clips leg (0: skip)")
    ap.add_argument("--stream-leg-seconds", type=int, default=600,
                    help="length of the configs[3] stream leg of the default run (0: skip)")
    ap.add_argument("--no-p32", action="store_true", help="skip the P32-coder extra measurement")
    ap.add_argument("--stream-steps", type=int, default=1)
    ap.add_argument("--stream-shard", action="store_true",
                    help="configs[3]: one 4K stream sharded over the GPUs with the RCCL gather (strong scaling)")
    ap.add_argument("--stream-seconds", type=int, default=600)
    ap.add_argument("--stream-mb", type=int, nargs=2, default=(240, 135))
    args = ap.parse_args()
    if args.stream_shard:
        return main_stream_shard(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    import avrecode_amd as avr
    from avrecode_amd.batch import DeviceBatch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = _local_device()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        _init_dist(world, dev)

    def barrier():
        if world > 1:
            dist.barrier()

    ctx = avr.Context(local)
    progress("generating the batch")
    data = make_input(ctx, args.slices, rank, args)
    ps = avr.parse_stream(data)
    assert len(ps.descs) == args.slices
    batch = DeviceBatch(ctx, ps)
    stream = torch.cuda.Stream(dev)
    mk = lambda: [torch.cuda.Event(enable_timing=True) for _ in range(4)]  # noqa: E731

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            batch.roundtrip_timed(mk(), avr.MODEL_PARALLEL, stream)
        stream.synchronize()
        verdict = batch.verdicts()
        bit_exact = bool((verdict == 1).all())
        res_c = batch.results("c")
        S = int(ps.descs["payload_size"].sum())
        C = int(res_c["out_len"][verdict == 1].sum())
        bins = int(res_c["bins"].sum())

        progress("warm-up done; timing")
        evs = [mk() for _ in range(args.steps)]
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            batch.roundtrip_timed(evs[k], avr.MODEL_PARALLEL, stream)
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
    # the timed steps recomputed the same outputs: re-check them, and against the oracle's answer
    bit_exact = bit_exact and bool((batch.verdicts() == 1).all())
    gold = golden_check(batch, data, args) if rank == 0 else None
    if gold is not None and gold.get("match") is False:
        bit_exact = False
    t_comp = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps / 1e3
    t_dec = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps / 1e3
    # labelled extra, outside the headline's timed region: the same batch through the P32 coder
    p32 = None
    if world == 1 and not args.no_p32:
        p32 = p32_extra(batch, args, stream, mk, len(data), C)

    tot = torch.tensor([elapsed, len(data), 0.0 if bit_exact else 1.0], dtype=torch.float64, device=_coll(dev))
    if world > 1:
        mx = tot[0:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot[1:3].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, total_bytes, bad = float(mx[0]), float(sm[0]), float(sm[1])
    else:
        total_bytes, bad = float(len(data)), float(tot[2])

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        dominant, t_dom = ("compress", t_comp) if t_comp >= t_dec else ("decompress", t_dec)
        kernel_name = ctx.slice_kernel(args.slices, ps.max_mb_width, dominant == "decompress")
        achieved = (S + C) / t_dom / 1e9
        line = {
            "metric": METRIC,
            "value": total_bytes * args.steps / elapsed / 1e6,
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device generator, seeded)",
            "bit_exact": bit_exact and bad == 0,
            "config": {
                "workload": WORKLOAD,
                "slices_per_gpu": args.slices,
                "mb": [args.mb_width, args.mb_height],
                "qp": list(QPS),
                "model": "parallel (the reference model reset per slice, SURVEY.md 7)",
                "coder": "arithmetic_code<uint64_t,uint8_t> (the reference's: 64-bit interval, byte digits, "
                         "p1 = (range / (pos + neg)) * pos exact; arithmetic_code.h:106-126, 232-248)",
                "input_bytes_per_gpu": len(data),
                "payload_bytes_S": S,
                "recoded_bytes_C": C,
                "bins": bins,
                "compress_ms": t_comp * 1e3,
                "decompress_ms": t_dec * 1e3,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel_name,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_traffic(args, kernel_name),
            },
            "cpu_baseline": None,
        }
        if gold is not None:
            line["oracle_parity"] = gold
        if p32 is not None:
            line["p32"] = p32
        progress(f"batch: {line['value']:.1f} MB/s")
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(ctx, args, len(data))
            progress("cpu baseline done")
        if world == 1 and not args.no_files:
            line["file_roundtrip"] = file_roundtrips(ctx, args)
        if world == 1 and not args.no_corpus:
            line["corpus"] = corpus_section(ctx, args)
        if world == 1 and args.rfiles > 0 and not args.no_files:
            line["rmode_files"] = rmode_files_section(ctx, args)
        if world == 1 and args.rclips > 0 and not args.no_files:
            line["rmode_clips"] = rmode_clips_section(ctx, args)
    if world > 1 and not args.no_corpus:
        rec = corpus_sharded(ctx, args, world, rank, dev)
        if rank == 0:
            line["corpus"] = rec
    # BASELINE configs[3] at its full length (600 s of 4K, 18,000 slices) as a labelled extra key:
    # at N = 1 beside the headline, at N > 1 sharded over the ranks (strong scaling; the only
    # leg with a data-path collective: the gathers and the scatter over RCCL)
    if args.stream_leg_seconds > 0 and not args.no_files:
        _init_dist(world, dev)
        try:
            rec = stream_shard_leg(ctx, args, args.stream_leg_seconds, world, rank, dev,
                                   with_cpu=world == 1 and not args.no_cpu_baseline)
        except Exception as e:   # the headline stands without this leg
            progress(f"rank {rank}: stream leg failed: {e!r}")
            rec = {"error": repr(e)[:500]}
        if rank == 0:
            line["stream_shard"] = rec
            if "value" in rec:
                progress(f"stream leg: {rec['value']:.1f} MB/s")
    if rank == 0:
        emit(line)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    # Native libraries (RCCL prints its version banner at init) write to file descriptor 1: point it
    # at stderr and keep the original stdout for the one JSON line.
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    main()
