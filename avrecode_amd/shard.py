"""Multi-GPU sharding: one process per GPU.

PARALLEL model, one file over the ranks, both directions.  Every slice is an independent unit
(fresh CABAC contexts per H.264 9.3.1, fresh re-coded coder per slice, recode.cpp:1263/1422, model
reset per slice), so a file's slices are cut into contiguous ranges balanced by bytes, one range
per rank.  The only collective is the final gather of the variable-length per-slice outputs to
rank 0 (point-to-point send/recv over xGMI with backend "nccl" = RCCL; CPU tensors with "gloo"):
  sharded_compress    re-coded blocks -> rank 0 builds the Recoded container (avr_assemble_container)
  sharded_decompress  regenerated CABAC payloads -> rank 0 splices them with the container's
                      literals and applies the last-byte patch (avr_splice_container)
Both are byte-identical to the single-GPU calls.

CHAINED model (the reference model restarted every AVR_CHAIN_SLICES coded slices), one file over
the ranks, both directions: its chains are independent, so a file's chains are cut into contiguous
ranges balanced by bytes (the library applies partition()'s rule), each rank runs its chains on its
GPU (avr_compress_chain_range / avr_decompress_chain_range), and the same gather brings the
re-coded (regenerated) slices to rank 0, which assembles (splices) them:
  sharded_compress_chained / sharded_decompress_chained: byte-identical to ctx.compress(data,
  MODEL_CHAINED) / ctx.decompress(avrc).

A corpus of files (BASELINE configs[4]): files are dealt to ranks whole (deal_files, LPT by
bytes) and each rank runs its files through the batched corpus calls; the reference model's
unit of sequential work is a file (its estimators carry across slices, recode.cpp:662-665), so
this is also the reference model's only split -- replicas over files.
"""
from __future__ import annotations

import numpy as np

from . import (MODEL_CHAINED, MODEL_PARALLEL, DecompressPlan, ParsedStream, assemble_container, container_model,
               parse_stream, plan_decompress, splice_container)


def partition(sizes, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) slice ranges, one per rank, balanced by cumulative bytes.

    Rank r takes the slices whose byte-prefix midpoint falls in [r, r+1) * total / world, so
    every slice is owned exactly once and ranges are ordered by rank."""
    sizes = np.asarray(sizes, dtype=np.float64)
    n = len(sizes)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    total = sizes.sum()
    if total <= 0:
        cuts = [round(r * n / world) for r in range(world + 1)]
    else:
        mid = np.cumsum(sizes) - sizes / 2
        owner = np.minimum((mid * world / total).astype(np.int64), world - 1)
        cuts = [int(np.searchsorted(owner, r, side="left")) for r in range(world)] + [n]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def pinned(nbytes: int):
    """A page-locked host buffer (uint8 numpy view of a pinned torch tensor): device copies into and
    out of it run as DMA at the link's rate, and one allocation is reused from step to step (a
    fresh multi-GB numpy array costs its page faults on every step)."""
    import torch
    t = torch.empty(max(1, nbytes), dtype=torch.uint8, pin_memory=True)
    return t.numpy()


def gather_flat(flat, status, offsets, lens, dst: int = 0, device=None, out=None):
    """Gather every rank's per-slice (status, bytes) to `dst`, in rank order.

    flat: this rank's outputs packed in one uint8 tensor (device tensor with RCCL), slice k's bytes
    at flat[offsets[k] : offsets[k] + lens[k]].  Returns (status int32[n_total], blob uint8 array,
    offsets uint64, lens uint32) on dst, None elsewhere.  The blob is one host array written in
    place (out: a caller's buffer of at least the total size, ideally pinned(): reused across steps,
    copied into by DMA); a multi-GB gather is copied once, device to host.  Counts first (a
    fixed-size all_gather), then one send/recv of the per-slice metadata and one of the flat bytes
    per rank: RCCL has no gatherv, and the payload moves device to device over xGMI.
    On dst the receives are posted for all ranks at once (each peer's xGMI link carries its own)
    and each rank's bytes go to the host on a copy stream as soon as they have arrived, while the
    later ranks' are still in flight."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    dev = device if device is not None else flat.device
    status = np.asarray(status, dtype=np.int64)
    offsets = np.asarray(offsets, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    n = len(status)
    nbytes = int((offsets + lens).max()) if n else 0
    hdr = torch.tensor([n, nbytes], dtype=torch.int64, device=dev)
    allh = [torch.zeros_like(hdr) for _ in range(world)]
    dist.all_gather(allh, hdr)
    counts = [int(h[0]) for h in allh]
    sizes = [int(h[1]) for h in allh]
    meta = torch.from_numpy(np.concatenate([status, offsets, lens])).to(dev)
    body = flat[:nbytes].to(dev)
    if rank != dst:
        if counts[rank]:
            dist.send(meta, dst)
        if sizes[rank]:
            dist.send(body, dst)
        return None
    total = sum(sizes)
    if out is not None and out.nbytes >= total:
        blob = out[:total]
    else:
        blob = np.empty(total, dtype=np.uint8)
    # post every receive, then drain them in rank order
    bufs, works = [], []
    for r in range(world):
        if r == rank:
            bufs.append((meta, body))
            continue
        m = torch.empty(3 * counts[r], dtype=torch.int64, device=dev)
        f = torch.empty(sizes[r], dtype=torch.uint8, device=dev)
        if counts[r]:
            works.append(dist.irecv(m, r))
        if sizes[r]:
            works.append(dist.irecv(f, r))
        bufs.append((m, f))
    on_gpu = dev.type == "cuda"
    copy_stream = torch.cuda.Stream(dev) if on_gpu else None
    st, offs, ln, base, wi = [], [], [], 0, 0
    for r in range(world):
        m, f = bufs[r]
        if r != rank:
            for _ in range(int(counts[r] > 0) + int(sizes[r] > 0)):
                works[wi].wait()
                wi += 1
        c = counts[r]
        if sizes[r]:
            dst_t = torch.from_numpy(blob[base:base + sizes[r]])
            if on_gpu:
                # after the receive (waited on the current stream), on the copy stream: this rank's
                # D2H overlaps the next ranks' receives
                copy_stream.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(copy_stream):
                    dst_t.copy_(f, non_blocking=dst_t.is_pinned())
                    f.record_stream(copy_stream)
            else:
                dst_t.copy_(f)
        mh = m.cpu().numpy()
        st.append(mh[:c])
        offs.append(mh[c:2 * c] + base)
        ln.append(mh[2 * c:])
        base += sizes[r]
    if on_gpu:
        copy_stream.synchronize()
    cat = lambda xs, t: np.concatenate(xs).astype(t) if xs else np.zeros(0, t)  # noqa: E731
    return cat(st, np.int32), blob, cat(offs, np.uint64), cat(ln, np.uint32)


def gather_blocks(local: list[bytes], status: list[int], dst: int = 0, device=None, out=None):
    """gather_flat for host byte strings (one per slice)."""
    import torch
    lens = np.array([len(b) for b in local], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if len(lens) else lens
    flat = torch.from_numpy(np.frombuffer(b"".join(local), dtype=np.uint8).copy())
    dev = device if device is not None else torch.device("cpu")
    return gather_flat(flat, status, offs, lens, dst=dst, device=dev, out=out)


def subset(ps: ParsedStream, lo: int, hi: int, copy_arena: bool = True) -> ParsedStream:
    """The slices [lo, hi) of a parsed stream as a self-contained batch (offsets rebased).
    copy_arena False: the arena is a view of ps.arena's range (valid while ps.arena is)."""
    d = ps.descs[lo:hi].copy()
    if len(d) == 0:
        return ParsedStream(d, np.zeros(16, np.uint8), 0, ps.max_mb_width, ps.max_mb_height)
    a0 = int(d[0]["payload_offset"])
    a1 = int(ps.descs[hi]["payload_offset"]) if hi < len(ps.descs) else len(ps.arena)
    w0 = int(d[0]["out_offset"])
    w1 = int(d[-1]["out_offset"]) + ((int(d[-1]["out_capacity"]) + 15) & ~15)
    d["payload_offset"] -= a0
    d["out_offset"] -= w0
    arena = ps.arena[a0:a1]
    return ParsedStream(d, arena.copy() if copy_arena else arena, w1 - w0, ps.max_mb_width, ps.max_mb_height)


def sharded_compress(ctx, data: bytes, device=None, ps: ParsedStream | None = None,
                     model: int = MODEL_PARALLEL) -> bytes | None:
    """PARALLEL-model compress of one file across all ranks; the container is returned on rank 0.

    Every rank parses the file (host), takes its contiguous slice range (partition), runs it on its
    GPU (compress + device roundtrip check: a slice is coded only if it regenerates its payload),
    packs the re-coded bytes on the device and sends them to rank 0 (gather_flat over RCCL), which
    assembles the Recoded container from its own parse (avr_assemble_container_parsed).
    Byte-identical to ctx.compress(data, model); model = MODEL_PARALLEL or MODEL_PARALLEL32."""
    import torch
    import torch.distributed as dist

    from .batch import DeviceBatch

    rank, world = dist.get_rank(), dist.get_world_size()
    ps = ps if ps is not None else parse_stream(data)
    lo, hi = partition(ps.descs["payload_size"], world)[rank]
    part = subset(ps, lo, hi)
    dev = _gather_device(ctx, device)
    if hi > lo:
        b = DeviceBatch(ctx, part)
        b.roundtrip(model)
        flat, d_off = b.pack()
        torch.cuda.synchronize()
        v = b.verdicts()
        res = b.results("c")
        offs = d_off.cpu().numpy()[: hi - lo].astype(np.int64)
        lens = np.where(res["status"] == 0, res["out_len"], 0).astype(np.int64)
        status = np.where(v == 1, 0, -1).astype(np.int64)
    else:
        import torch as _t
        flat = _t.zeros(16, dtype=_t.uint8, device=dev)
        offs = lens = status = np.zeros(0, np.int64)
    g = gather_flat(flat, status, offs, lens, dst=0, device=dev)
    if g is None:
        return None
    st, blob, offs, lens = g
    return assemble_container(data, st, blob, offs, lens, model=model, ps=ps)


def _gather_device(ctx, device):
    import torch
    import torch.distributed as dist
    # RCCL ("nccl") moves device tensors only; gloo moves host tensors
    if dist.get_backend() == "nccl":
        return device if device is not None else torch.device("cuda", ctx.device)
    return torch.device("cpu")


def decompress_range(ctx, part: ParsedStream, device=None, model: int = MODEL_PARALLEL):
    """This rank's slice range of a sharded decompress on its GPU: (flat uint8 tensor, status,
    offsets, lens) with slice k's regenerated bytes at flat[offsets[k] : offsets[k] + lens[k]]
    (packed on the device, avr_pack_outputs).  model: the container's (container_model)."""
    import torch

    from .batch import DeviceBatch

    b = DeviceBatch(ctx, part, device=device)
    b.decompress(model)
    flat, d_off = b.pack(which="d")
    torch.cuda.synchronize()
    res = b.results("d")
    n = len(part.descs)
    offs = d_off.cpu().numpy()[:n].astype(np.int64)
    status = res["status"].astype(np.int64)
    lens = np.where(status == 0, res["out_len"], 0).astype(np.int64)
    return flat, status, offs, lens


def sharded_decompress(ctx, avrc: bytes, device=None, run_range=None) -> bytes | None:
    """PARALLEL-model decompress of one container across all ranks; the file is returned on rank 0.

    Every rank plans the container (host: avr_plan_decompress), takes its contiguous range of
    coded slices balanced by re-coded bytes (partition), regenerates them on its GPU
    (decompress_range: avr_decompress_slices + avr_pack_outputs), and sends the packed payloads to
    rank 0 (gather_flat over RCCL), which splices them with the literals and applies the last-byte
    patch (avr_splice_container, recode.cpp:1338-1357).  Byte-identical to ctx.decompress(avrc).
    run_range(part) -> (flat, status, offsets, lens) replaces the device step (CPU tests)."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    plan = plan_decompress(avrc)
    model = container_model(avrc)
    lo, hi = partition(plan.descs["payload_size"], world)[rank]
    part = subset(plan, lo, hi)
    dev = _gather_device(ctx, device)
    if hi > lo:
        flat, status, offs, lens = (run_range or (lambda p: decompress_range(ctx, p, device, model)))(part)
    else:
        flat = torch.zeros(16, dtype=torch.uint8, device=dev)
        offs = lens = status = np.zeros(0, np.int64)
    g = gather_flat(flat, status, offs, lens, dst=0, device=dev)
    if g is None:
        return None
    st, blob, offs, lens = g
    return splice_container(avrc, st, blob, offs, lens)


def _host_to_gather(blob, dev):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(blob) if len(blob) else np.zeros(16, np.uint8))
    return t.to(dev) if dev.type == "cuda" else t


def sharded_compress_chained(ctx, data, device=None, run_range=None) -> bytes | None:
    """CHAINED-model compress of one file across all ranks; the container is returned on rank 0.

    Every rank runs its contiguous range of the file's chains on its GPU
    (Context.compress_chain_range: parse and segmentation of the whole file, the reference-model
    pass over its chains), the re-coded slices go to rank 0 (gather_flat over RCCL), which assembles
    the Recoded container (avr_assemble_container, model CHAINED).  Byte-identical to
    ctx.compress(data, MODEL_CHAINED).  A coded slice that failed on its rank (status -2: the
    whole-file call would demote it and re-segment, moving every later chain) makes rank 0 compress
    the file whole.  run_range() -> compress_chain_range's tuple replaces the device step (tests)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    dev = _gather_device(ctx, device)
    lo, hi, st, blob, offs, lens = (run_range or (lambda: ctx.compress_chain_range(data, world, rank)))()
    g = gather_flat(_host_to_gather(blob, dev), st.astype(np.int64), offs.astype(np.int64), lens.astype(np.int64),
                    dst=0, device=dev)
    if g is None:
        return None
    st, blob, offs, lens = g
    if (st < -1).any():
        return ctx.compress(data, MODEL_CHAINED)
    return assemble_container(data, st, blob, offs, lens, model=MODEL_CHAINED)


def sharded_decompress_chained(ctx, avrc, device=None, run_range=None) -> bytes | None:
    """CHAINED-model decompress of one container across all ranks; the file is returned on rank 0.

    Every rank plans the container and regenerates its contiguous range of chains on its GPU
    (Context.decompress_chain_range); the regenerated slices go to rank 0 (gather_flat), which
    splices them with the literals and the last-byte patch on its plan of the same container
    (DecompressPlan.splice, recode.cpp:1338-1357).  Byte-identical to ctx.decompress(avrc).
    A reference-model container is one unit: rank 0 decodes it whole."""
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    dev = _gather_device(ctx, device)
    lo, hi, st, regen, offs, lens = (run_range or (lambda: ctx.decompress_chain_range(avrc, world, rank)))()
    g = gather_flat(_host_to_gather(regen, dev), st.astype(np.int64), offs.astype(np.int64), lens.astype(np.int64),
                    dst=0, device=dev)
    if g is None:
        return None
    st, blob, offs, lens = g
    out = DecompressPlan().load(avrc).splice(st, blob, offs, lens)
    return out.tobytes()


def scatter_parsed(ps: "ParsedStream | None", ranges, device, src: int = 0):
    """Rank src's decompress batch (ps, e.g. DecompressPlan.parsed of the container it assembled) cut
    into the contiguous slice ranges `ranges` (one [lo, hi) per rank): each rank receives its own as
    (descs, arena, n, work_len, max_mb_width, max_mb_height) -- host arrays on src, the arena as a
    device tensor elsewhere (point-to-point over RCCL / xGMI: one header, the descriptors and the
    re-coded streams per rank; gloo moves host tensors).  Offsets are rebased as in subset()."""
    import torch
    import torch.distributed as dist

    from . import SLICE_DESC

    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == src:
        mine = None
        pending = []   # every rank's messages in flight at once (each peer has its own xGMI link)
        for r in range(world):
            lo, hi = ranges[r]
            sub = ps if (lo, hi) == (0, len(ps.descs)) else subset(ps, lo, hi, copy_arena=r == rank)
            if r == rank:
                mine = sub
                continue
            hdr = torch.tensor([hi - lo, sub.arena.nbytes, sub.work_len, sub.max_mb_width, sub.max_mb_height],
                               dtype=torch.int64, device=device)
            msgs = [hdr]
            if hi > lo:
                # the arena range is a view of rank src's (pinned) arena: one DMA to the device
                msgs.append(torch.from_numpy(np.ascontiguousarray(sub.descs).view(np.uint8).reshape(-1)).to(device))
                msgs.append(torch.from_numpy(sub.arena).to(device, non_blocking=True))
            for t in msgs:
                pending.append((dist.isend(t, r), t))
        for w, _ in pending:
            w.wait()
        return (mine.descs, mine.arena, len(mine.descs), mine.work_len, mine.max_mb_width, mine.max_mb_height)
    hdr = torch.zeros(5, dtype=torch.int64, device=device)
    dist.recv(hdr, src)
    n, alen, wlen, mw, mh = (int(x) for x in hdr.cpu())
    descs = np.zeros(0, dtype=SLICE_DESC)
    arena = torch.zeros(16, dtype=torch.uint8, device=device)
    if n:
        d = torch.empty(n * SLICE_DESC.itemsize, dtype=torch.uint8, device=device)
        dist.recv(d, src)
        descs = d.cpu().numpy().view(SLICE_DESC)
        arena = torch.empty(alen, dtype=torch.uint8, device=device)
        dist.recv(arena, src)
    return descs, arena, n, wlen, mw, mh


def deal_files(sizes, world: int) -> list[list[int]]:
    """Files to ranks, whole: longest-processing-time-first by bytes (the largest file goes to the
    least-loaded rank).  Returns each rank's file indices in ascending order."""
    sizes = [int(x) for x in sizes]
    load = [0] * max(1, world)
    owned = [[] for _ in range(max(1, world))]
    for f in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        r = min(range(len(load)), key=lambda q: (load[q], q))
        load[r] += sizes[f]
        owned[r].append(f)
    return [sorted(o) for o in owned]


def corpus_roundtrip(ctx, files: list[bytes], model: int, dst: int = 0):
    """A corpus over the ranks (BASELINE configs[4]): this rank's files (deal_files) compressed
    and decompressed as one batch each (avr_compress_files / avr_decompress_files) and checked
    byte for byte.  Returns (files done here, bytes in, container bytes, all files bit-exact here);
    the callers reduce these over ranks."""
    rank, world = _rank_world()
    mine = deal_files([len(f) for f in files], world)[rank]
    if not mine:
        return 0, 0, 0, True
    sub = [files[i] for i in mine]
    comp = ctx.compress_files(sub, model)
    ok = not any(isinstance(c, Exception) for c in comp)
    dec = ctx.decompress_files([c for c in comp if not isinstance(c, Exception)]) if ok else []
    ok = ok and all(not isinstance(d, Exception) and d == f for d, f in zip(dec, sub))
    return len(sub), sum(map(len, sub)), sum(len(c) for c in comp if not isinstance(c, Exception)), ok


def _rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1
