"""Host halves of the sharded configs[3] roundtrip (CPU, no GPU compute):

* rank 0's container assembly into a reused caller buffer (avr_assemble_container_into) gives the
  golden containers, and refuses a buffer that is too small with the size it needs;
* the decompress plan handle (avr_dec_plan_*: decompressor::run's read_packet parse, the arena of
  re-coded streams, the splice with the literals and the last-byte patch, recode.cpp:1338-1409)
  equals avr_plan_decompress / avr_splice_container, across reloads of one handle;
* shard.scatter_parsed hands every rank exactly shard.subset of rank 0's plan (gloo, world 2 and 3);
* the parse's payloads of NAL units with emulation-prevention bytes equal a plain restatement of
  7.4.1's unescaping, and the positions it reports for verbatim payloads are theirs in the file;
* assembly of a stream of the configs[3] shape runs at memory speed (reported; a loose floor only).
"""
import hashlib
import json
import os
import tempfile
import time

import numpy as np
import pytest

from _oracle import ROOT, slices_p

import avrecode_amd as avr
from avrecode_amd import shard

FIX = ROOT / "tests" / "fixtures"
GOLD = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}


def _oracle_outputs(data, p32=False):
    _, recs = slices_p(data, p32=p32)
    st = np.array([0 if r["recodable"] else -1 for r in recs], np.int32)
    blobs = [r["recoded"] if r["recodable"] else b"" for r in recs]
    lens = np.array([len(b) for b in blobs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    return st, b"".join(blobs), offs, lens


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_assemble_into_caller_buffer(name):
    data = (FIX / name).read_bytes()
    ps = avr.parse_stream(data)
    st, blob, offs, lens = _oracle_outputs(data)
    bound = avr.container_bound(len(data), len(st), int(lens.sum()))
    buf = np.full(bound, 0xEE, np.uint8)
    for _ in range(2):   # the same buffer twice: a step reuses it
        c = avr.assemble_container(data, st, blob, offs, lens, ps=ps, out=buf)
        assert hashlib.sha256(c.tobytes()).hexdigest() == GOLD[(name, "P")]["avrc_sha256"]
    assert c.tobytes() == avr.assemble_container(data, st, blob, offs, lens, ps=ps)
    with pytest.raises(avr.AvrError) as e:
        avr.assemble_container(data, st, blob, offs, lens, ps=ps, out=np.empty(len(c) - 1, np.uint8))
    assert str(len(c)) in str(e.value)


def _container_payloads(data: bytes, avrc: bytes) -> list[bytes]:
    desc, _ = avr.describe_container(avrc)
    pos, out = 0, []
    for b in desc["blocks"]:
        if "literal" in b:
            pos += len(bytes.fromhex(b["literal"]))
        elif "cabac" in b:
            out.append(data[pos:pos + b["size"]])
            pos += b["size"]
    return out


def test_dec_plan_handle_equals_plan_and_splice():
    from _oracle import oracle_cli
    h = avr.DecompressPlan()
    for name in ("realshort.mp4", "cockatoo.mp4", "realshort.mp4"):   # one handle, reloaded
        data = (FIX / name).read_bytes()
        avrc = oracle_cli("compress", FIX / name, mode="P")
        ref = avr.plan_decompress(avrc)
        h.load(avrc)
        arena = np.full(h.arena_len + 64, 0xAB, np.uint8)
        pp = h.parsed(arena)
        assert pp.descs.tobytes() == ref.descs.tobytes()
        assert pp.arena.tobytes() == ref.arena.tobytes()
        assert (pp.work_len, pp.max_mb_width, pp.max_mb_height) == (ref.work_len, ref.max_mb_width, ref.max_mb_height)
        pays = _container_payloads(data, avrc)
        lens = np.array([len(p) for p in pays], np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        st = np.zeros(len(pays), np.int32)
        regen = b"".join(pays)
        out = np.zeros(len(data) + 100, np.uint8)
        f = h.splice(st, regen, offs, lens, out=out)
        assert f.tobytes() == data == avr.splice_container(avrc, st, regen, offs, lens)
        assert h.splice(st, regen, offs, lens).tobytes() == data
        with pytest.raises(avr.AvrError):
            h.splice(st, regen, offs, lens, out=np.zeros(len(data) - 1, np.uint8))
        with pytest.raises(avr.AvrError):
            h.splice(st, regen[:-1], offs, lens)
        st[len(st) // 2] = -9
        with pytest.raises(avr.AvrError):
            h.splice(st, regen, offs, lens)
    # a reference- or chained-model container plans every slice, coded or not (the reference
    # model turns frames over on uncoded ones): the indexing of avr_decompress_chain_range's outputs
    data = (FIX / "realshort.mp4").read_bytes()
    for mode in ("R", "C"):
        assert h.load(oracle_cli("compress", FIX / "realshort.mp4", mode=mode)).n_slices == len(avr.parse_stream(data).descs)
    with pytest.raises(avr.AvrError) as e:   # the one-shot slice batch stays parallel-model only
        avr.plan_decompress(oracle_cli("compress", FIX / "realshort.mp4", mode="C"))
    assert e.value.code == -6
    h.close()


def _scatter_worker(rank, world, port, outdir):
    import torch.distributed as dist
    from _oracle import oracle_cli
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        avrc = oracle_cli("compress", FIX / "cockatoo.mp4", mode="P")
        plan = avr.plan_decompress(avrc)   # every rank: the expected parts
        ranges = shard.partition(plan.descs["payload_size"], world)
        import torch
        pp = None
        if rank == 0:
            h = avr.DecompressPlan().load(avrc)
            pp = h.parsed()
        descs, arena, n, wl, mw, mh = shard.scatter_parsed(pp, ranges if rank == 0 else None, torch.device("cpu"))
        lo, hi = ranges[rank]
        want = shard.subset(plan, lo, hi)
        arena = arena if isinstance(arena, np.ndarray) else arena.numpy()
        ok = (n == hi - lo and descs.tobytes() == want.descs.tobytes() and wl == want.work_len and
              arena.tobytes() == want.arena.tobytes() and (mw, mh) == (want.max_mb_width, want.max_mb_height))
        with open(os.path.join(outdir, f"{rank}.ok"), "w") as f:
            f.write("1" if ok else "0")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_scatter_parsed(world):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_scatter_worker, args=(world, port, td), nprocs=world, join=True)
        assert all(open(os.path.join(td, f"{r}.ok")).read() == "1" for r in range(world))


def _unescape(raw: bytes) -> bytes:
    """7.4.1, as written: every 00 00 03 drops its 03."""
    out, i = bytearray(), 0
    while i < len(raw):
        if i + 2 < len(raw) and raw[i] == 0 and raw[i + 1] == 0 and raw[i + 2] == 3:
            out += b"\x00\x00"
            i += 3
        else:
            out.append(raw[i])
            i += 1
    return bytes(out)


def test_parse_payloads_and_file_positions():
    import test_assembly_scaling as t
    data = t._stream(60, 9)
    ps = avr.parse_stream(data)
    head, nals = t._nals(data)
    slices = [n for n in nals if (n[4] & 0x1F) in (1, 5)]
    assert len(slices) == len(ps.descs) == 60
    n_verbatim = 0
    for d, nal in zip(ps.descs, slices):
        o, m = int(d["payload_offset"]), int(d["payload_size"])
        pay = ps.arena[o:o + m].tobytes()
        rbsp = _unescape(nal[5:])
        assert pay in rbsp
        fo = int(d["file_offset"])
        if fo != (1 << 64) - 1:
            n_verbatim += 1
            assert data[fo:fo + m] == pay and _unescape(nal[5:]) == nal[5:]
        else:
            assert _unescape(nal[5:]) != nal[5:]
    assert 0 < n_verbatim < 60


def test_assembly_rate_at_stream_scale():
    """~1 GB stream of 4,000 slices of ~250 KB (the 4K stream's slice size; payloads without
    emulation-prevention bytes, as most of the generator's), assembled into a reused buffer: the
    rate is printed; the floor is loose (shared CI hosts)."""
    import test_assembly_scaling as t
    head, sl = t._nals(t._stream(30, 4))
    # payloads ~250 KB: one slice NAL template with random bytes appended
    rng = np.random.default_rng(1)
    tmpl = sl[2][:64]
    big = []
    for i in range(40):
        raw = rng.integers(1, 256, size=250_000, dtype=np.uint8).tobytes()
        big.append(tmpl + raw + b"\x80")
    data = head + b"".join(big) * 100   # 4,000 slices, ~1 GB
    ps = avr.parse_stream(data)
    n = len(ps.descs)
    assert n == 4000
    st = np.zeros(n, np.int32)
    lens = (ps.descs["payload_size"] * 0.99).astype(np.uint32)   # stand-in re-coded sizes
    offs = ps.descs["payload_offset"].astype(np.uint64)
    buf = np.empty(avr.container_bound(len(data), n, int(lens.sum())), np.uint8)
    avr.assemble_container(data, st, ps.arena, offs, lens, ps=ps, out=buf)   # maps the buffer
    t0 = time.perf_counter()
    c = avr.assemble_container(data, st, ps.arena, offs, lens, ps=ps, out=buf)
    dt = time.perf_counter() - t0
    rate = len(data) / dt / 1e9
    print(f"assembly: {len(data) / 1e9:.2f} GB in {dt:.3f} s = {rate:.2f} GB/s")
    assert len(c) > len(data) * 0.98
    assert rate > 0.3


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4", "paff_ipp.264"])
def test_parse_range_equals_subset(name):
    """A rank's own range of a stream (avr_parse_stream_range) is shard.subset of the whole parse,
    and avr_slice_payload_sizes the whole parse's payload sizes: the other ranks of a sharded run
    need neither the whole arena nor a copy of every payload."""
    data = (FIX / name).read_bytes()
    ps = avr.parse_stream(data)
    n = len(ps.descs)
    assert (avr.slice_payload_sizes(data) == ps.descs["payload_size"]).all()
    for lo, hi in ((0, n), (0, n // 2), (n // 3, n), (n // 2, n // 2), (1, 2)):
        a, b = avr.parse_stream(data, lo, hi), shard.subset(ps, lo, hi)
        assert a.descs.tobytes() == b.descs.tobytes(), (lo, hi)
        if hi > lo:
            assert a.arena.tobytes()[:len(b.arena)] == b.arena.tobytes()
        assert a.work_len == b.work_len


@pytest.mark.parametrize("name", ["paff_ipp.264", "mbaff_ib.264"])
def test_dec_plan_of_annexb_containers(name):
    """An Annex-B container's plan (decompressor::run's read_packet parse, recode.cpp:1338-1409):
    the surrogate fills are stepped over by the start-code scan and the emulation-prevention check
    (avr_front SkipRanges), and the slices it finds carry the headers of the original file's coded
    slices, in order; the splice restores the file."""
    from _oracle import oracle_cli
    import test_assembly_scaling as tas
    data = (FIX / name).read_bytes()
    ps = avr.parse_stream(data)
    avrc = oracle_cli("compress", FIX / name, mode="P")
    h = avr.DecompressPlan().load(avrc)
    mine = [k for k, f in enumerate(tas._layout_of(avrc)) if f is not None]   # the coded slices
    assert len(mine) == h.n_slices > 0
    hdr = ("slice_type", "slice_qp", "cabac_init_idc", "first_mb", "mb_width", "mb_height", "picture_id",
           "structure", "transform_8x8_mode", "num_ref_idx_l0", "num_ref_idx_l1")
    for j, k in enumerate(mine):
        for f in hdr:
            assert h.descs[j][f] == ps.descs[k][f], (name, j, k, f)
    pays = _container_payloads(data, avrc)
    lens = np.array([len(p) for p in pays], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    assert h.splice(np.zeros(len(pays), np.int32), b"".join(pays), offs, lens).tobytes() == data
