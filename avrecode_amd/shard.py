"""Multi-GPU sharding of the PARALLEL model: one process per GPU.

Every slice is an independent unit in the parallel model (fresh CABAC contexts per H.264 9.3.1,
fresh re-coded coder per slice, recode.cpp:1263/1422, model reset per slice), so a file's slices
are cut into contiguous ranges balanced by payload bytes, one range per rank.  The only
collective is the final gather of the variable-length re-coded blocks to rank 0 (point-to-point
send/recv over xGMI with backend "nccl" = RCCL; CPU tensors with "gloo"), where the host builds
the Recoded container (avr_assemble_container).  The reference model has no such split: its
estimators carry across slices (recode.cpp:662-665), so it runs as replicas only.
"""
from __future__ import annotations

import numpy as np

from . import MODEL_PARALLEL, ParsedStream, assemble_container, parse_stream


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


def gather_flat(flat, status, offsets, lens, dst: int = 0, device=None):
    """Gather every rank's per-slice (status, bytes) to `dst`, in rank order.

    flat: this rank's outputs packed in one uint8 tensor (device tensor with RCCL), slice k's bytes
    at flat[offsets[k] : offsets[k] + lens[k]].  Returns (status int32[n_total], blob bytes,
    offsets uint64, lens uint32) on dst, None elsewhere.  Counts first (a fixed-size all_gather),
    then one send/recv of the per-slice metadata and one of the flat bytes per rank: RCCL has no
    gatherv, and the payload moves device to device over xGMI."""
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
    st, offs, ln, blobs, base = [], [], [], [], 0
    for r in range(world):
        if r == rank:
            m, f = meta, body
        else:
            m = torch.empty(3 * counts[r], dtype=torch.int64, device=dev)
            f = torch.empty(sizes[r], dtype=torch.uint8, device=dev)
            if counts[r]:
                dist.recv(m, r)
            if sizes[r]:
                dist.recv(f, r)
        m = m.cpu().numpy()
        c = counts[r]
        st.append(m[:c])
        offs.append(m[c:2 * c] + base)
        ln.append(m[2 * c:])
        blobs.append(f.cpu().numpy().tobytes())
        base += sizes[r]
    cat = lambda xs, t: np.concatenate(xs).astype(t) if xs else np.zeros(0, t)  # noqa: E731
    return cat(st, np.int32), b"".join(blobs), cat(offs, np.uint64), cat(ln, np.uint32)


def gather_blocks(local: list[bytes], status: list[int], dst: int = 0, device=None):
    """gather_flat for host byte strings (one per slice)."""
    import torch
    lens = np.array([len(b) for b in local], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if len(lens) else lens
    flat = torch.from_numpy(np.frombuffer(b"".join(local), dtype=np.uint8).copy())
    dev = device if device is not None else torch.device("cpu")
    return gather_flat(flat, status, offs, lens, dst=dst, device=dev)


def subset(ps: ParsedStream, lo: int, hi: int) -> ParsedStream:
    """The slices [lo, hi) of a parsed stream as a self-contained batch (offsets rebased)."""
    d = ps.descs[lo:hi].copy()
    if len(d) == 0:
        return ParsedStream(d, np.zeros(16, np.uint8), 0, ps.max_mb_width, ps.max_mb_height)
    a0 = int(d[0]["payload_offset"])
    a1 = int(ps.descs[hi]["payload_offset"]) if hi < len(ps.descs) else len(ps.arena)
    w0 = int(d[0]["out_offset"])
    w1 = int(d[-1]["out_offset"]) + ((int(d[-1]["out_capacity"]) + 15) & ~15)
    d["payload_offset"] -= a0
    d["out_offset"] -= w0
    return ParsedStream(d, ps.arena[a0:a1].copy(), w1 - w0, ps.max_mb_width, ps.max_mb_height)


def sharded_compress(ctx, data: bytes, device=None, ps: ParsedStream | None = None) -> bytes | None:
    """PARALLEL-model compress of one file across all ranks; the container is returned on rank 0.

    Every rank parses the file (host), takes its contiguous slice range (partition), runs it on its
    GPU (compress + device roundtrip check: a slice is coded only if it regenerates its payload),
    packs the re-coded bytes on the device and sends them to rank 0 (gather_flat over RCCL), which
    assembles the Recoded container.  Byte-identical to ctx.compress(data, MODEL_PARALLEL)."""
    import torch
    import torch.distributed as dist

    from .batch import DeviceBatch

    rank, world = dist.get_rank(), dist.get_world_size()
    ps = ps if ps is not None else parse_stream(data)
    lo, hi = partition(ps.descs["payload_size"], world)[rank]
    part = subset(ps, lo, hi)
    # RCCL ("nccl") moves device tensors only; gloo moves host tensors
    if dist.get_backend() == "nccl":
        dev = device if device is not None else torch.device("cuda", ctx.device)
    else:
        dev = torch.device("cpu")
    if hi > lo:
        b = DeviceBatch(ctx, part)
        b.roundtrip(MODEL_PARALLEL)
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
    return assemble_container(data, st, blob, offs, lens)
