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


def gather_blocks(local: list[bytes], status: list[int], dst: int = 0, device=None):
    """Gather every rank's per-slice (status, bytes) to `dst`, in rank order.

    Returns (status int32[n_total], blob bytes, offsets uint64, lens uint32) on dst, None elsewhere.
    Sizes first (fixed-size all_gather of counts), then one send/recv of a flat byte tensor per
    rank: RCCL has no gatherv."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    dev = device if device is not None else torch.device("cpu")
    lens = np.array([len(b) for b in local], dtype=np.int64)
    hdr = torch.tensor([len(local), int(lens.sum())], dtype=torch.int64, device=dev)
    allh = [torch.zeros_like(hdr) for _ in range(world)]
    dist.all_gather(allh, hdr)
    counts = [int(h[0]) for h in allh]
    nbytes = [int(h[1]) for h in allh]
    meta = torch.from_numpy(np.concatenate([np.asarray(status, dtype=np.int64), lens])).to(dev)
    flat = torch.from_numpy(np.frombuffer(b"".join(local), dtype=np.uint8).copy()).to(dev)
    if rank != dst:
        if counts[rank]:
            dist.send(meta, dst)
        if nbytes[rank]:
            dist.send(flat, dst)
        return None
    statuses, blobs, all_lens = [], [], []
    for r in range(world):
        if r == rank:
            m, f = meta, flat
        else:
            m = torch.empty(2 * counts[r], dtype=torch.int64, device=dev)
            f = torch.empty(nbytes[r], dtype=torch.uint8, device=dev)
            if counts[r]:
                dist.recv(m, r)
            if nbytes[r]:
                dist.recv(f, r)
        m = m.cpu().numpy()
        statuses.append(m[: counts[r]])
        all_lens.append(m[counts[r]:])
        blobs.append(f.cpu().numpy().tobytes())
    st = np.concatenate(statuses).astype(np.int32) if statuses else np.zeros(0, np.int32)
    ln = np.concatenate(all_lens).astype(np.uint32) if all_lens else np.zeros(0, np.uint32)
    offs = np.concatenate([[0], np.cumsum(ln, dtype=np.uint64)[:-1]]).astype(np.uint64) if len(ln) else ln.astype(np.uint64)
    return st, b"".join(blobs), offs, ln


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


def sharded_compress(ctx, data: bytes, device=None) -> bytes | None:
    """PARALLEL-model compress of one file across all ranks; the container is returned on rank 0.

    Byte-identical to ctx.compress(data, MODEL_PARALLEL) on one GPU."""
    import torch
    import torch.distributed as dist

    from .batch import DeviceBatch

    rank, world = dist.get_rank(), dist.get_world_size()
    ps = parse_stream(data)
    lo, hi = partition(ps.descs["payload_size"], world)[rank]
    part = subset(ps, lo, hi)
    blobs, status = [], []
    if hi > lo:
        b = DeviceBatch(ctx, part)
        b.roundtrip(MODEL_PARALLEL)
        torch.cuda.synchronize()
        v = b.verdicts()
        rec = b.recoded()
        status = [0 if v[k] == 1 else -1 for k in range(hi - lo)]
        blobs = [rec[k] if v[k] == 1 else b"" for k in range(hi - lo)]
    # RCCL ("nccl") moves device tensors only; gloo moves host tensors
    if dist.get_backend() == "nccl":
        dev = device if device is not None else torch.device("cuda", ctx.device)
    else:
        dev = torch.device("cpu")
    g = gather_blocks(blobs, status, dst=0, device=dev)
    if g is None:
        return None
    st, blob, offs, lens = g
    return assemble_container(data, st, blob, offs, lens)
