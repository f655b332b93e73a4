"""CPU checks of the product's boundary and host logic (no GPU compute):

* libavrecode.so loads and exports every function include/avrecode.h declares;
* without a GPU the hot path fails loudly (no CPU fallback);
* avr_parse_stream hands the kernels the same slices/payloads the oracle decodes;
* avr_assemble_container, fed the oracle's per-slice outputs, reproduces the golden P-mode
  containers byte for byte (segmentation + protobuf);
* slice partitioning and the rank-0 gather (gloo, world_size 2) reassemble the same container.
"""
import hashlib
import json
import os
import re
import tempfile

import numpy as np
import pytest

from _oracle import ROOT, patch_restores, slices_p

import avrecode_amd as avr
from avrecode_amd import shard

FIX = ROOT / "tests" / "fixtures"
GOLD = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}


def test_library_exports_every_declared_symbol():
    header = (ROOT / "include" / "avrecode.h").read_text()
    declared = set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\**\s*(avr_\w+)\s*\(", header, re.M))
    assert declared == set(avr.EXPORTED_SYMBOLS)
    L = avr.lib()
    for name in declared:
        assert getattr(L, name) is not None


def test_no_gpu_means_loud_failure():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(avr.AvrError) as e:
        avr.Context(0)
    assert e.value.code == -2


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_parse_stream_agrees_with_oracle(name):
    data = (FIX / name).read_bytes()
    ps = avr.parse_stream(data)
    total, recs = slices_p(data)
    assert total == len(ps.descs)
    assert ps.max_mb_width > 0 and ps.work_len >= 2 * ps.payload_bytes
    for k, r in enumerate(recs):
        d = ps.descs[k]
        assert d["payload_offset"] % 16 == 0 and d["read_limit"] >= d["payload_size"]
        payload = ps.arena[int(d["payload_offset"]):int(d["payload_offset"]) + int(d["payload_size"])].tobytes()
        if r["recodable"]:
            assert d["coded"] == 1
            assert patch_restores(r["regen"], payload), k


def _oracle_outputs(data, p32=False):
    _, recs = slices_p(data, p32=p32)
    st = np.array([0 if r["recodable"] else -1 for r in recs], np.int32)
    return st, [r["recoded"] if r["recodable"] else b"" for r in recs]


@pytest.mark.parametrize("parsed", [False, True], ids=["reparse", "parsed"])
@pytest.mark.parametrize("mode", ["P", "P32"])
@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_assemble_container_matches_golden(name, mode, parsed):
    """Rank 0's assembly from the oracle's per-slice outputs gives the golden container of the
    mode (the u64 coder's "avrecode-amd:P64" or the P32 coder's "avrecode-amd:P32"), with the file
    parsed again or from the parse rank 0 already holds (avr_assemble_container_parsed)."""
    data = (FIX / name).read_bytes()
    st, blobs = _oracle_outputs(data, p32=mode == "P32")
    lens = np.array([len(b) for b in blobs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    model = avr.MODEL_PARALLEL32 if mode == "P32" else avr.MODEL_PARALLEL
    c = avr.assemble_container(data, st, b"".join(blobs), offs, lens, model=model,
                               ps=avr.parse_stream(data) if parsed else None)
    g = GOLD[(name, mode)]
    assert len(c) == g["avrc_len"] and hashlib.sha256(c).hexdigest() == g["avrc_sha256"]
    assert avr.container_model(c) == model


def test_assemble_container_rejects_bad_arguments():
    data = (FIX / "realshort.mp4").read_bytes()
    with pytest.raises(avr.AvrError):
        avr.assemble_container(data, np.zeros(3, np.int32), b"", np.zeros(3, np.uint64), np.zeros(3, np.uint32))
    with pytest.raises(avr.AvrError):
        avr.parse_stream(b"not a video")
    # a coded slice's bytes outside the gathered buffer, and the reference model (no assembly)
    st, blobs = _oracle_outputs(data)
    lens = np.array([len(b) for b in blobs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    blob = b"".join(blobs)
    with pytest.raises(avr.AvrError):
        avr.assemble_container(data, st, blob[:-1], offs, lens)
    with pytest.raises(avr.AvrError):
        avr.assemble_container(data, st, blob, offs, lens, model=avr.MODEL_REFERENCE)


def test_container_model_of_each_format():
    from _oracle import oracle_cli
    for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL), ("P32", avr.MODEL_PARALLEL32),
                        ("C", avr.MODEL_CHAINED)):
        assert avr.container_model(oracle_cli("compress", FIX / "realshort.mp4", mode=mode)) == model
    with pytest.raises(avr.AvrError):
        avr.container_model(b"\x0a\x10\x0a\x0eavrecode-amd:P")   # the round-2 format: refused
    assert avr.container_model(b"\x0a\x0c\x0a\x0aother:tag1") == avr.MODEL_REFERENCE   # a foreign tag


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_covers_and_balances(world):
    rng = np.random.default_rng(world)
    sizes = rng.integers(1, 100000, size=257)
    parts = shard.partition(sizes, world)
    assert len(parts) == world and parts[0][0] == 0 and parts[-1][1] == len(sizes)
    for (a, b), (c, d) in zip(parts, parts[1:]):
        assert b == c and a <= b
    loads = [sizes[a:b].sum() for a, b in parts]
    assert max(loads) <= sizes.sum() / world + sizes.max()
    assert shard.partition([], 4) == [(0, 0)] * 4


def test_subset_rebases_offsets():
    ps = avr.parse_stream((FIX / "realshort.mp4").read_bytes())
    sub = shard.subset(ps, 5, 9)
    assert len(sub.descs) == 4 and sub.descs[0]["payload_offset"] == 0 and sub.descs[0]["out_offset"] == 0
    for k in range(4):
        d0, d1 = ps.descs[5 + k], sub.descs[k]
        a = ps.arena[int(d0["payload_offset"]):int(d0["payload_offset"]) + int(d0["payload_size"])]
        b = sub.arena[int(d1["payload_offset"]):int(d1["payload_offset"]) + int(d1["payload_size"])]
        assert (a == b).all()
        assert int(d1["out_offset"]) + int(d1["out_capacity"]) <= sub.work_len


def _gloo_worker(rank, world, port, name, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = (FIX / name).read_bytes()
        ps = avr.parse_stream(data)
        lo, hi = shard.partition(ps.descs["payload_size"], world)[rank]
        _, recs = slices_p(data, lo, hi)          # stands in for this rank's device output
        st = [0 if r["recodable"] else -1 for r in recs]
        blobs = [r["recoded"] if r["recodable"] else b"" for r in recs]
        # at world 8, rank 0 gathers into a caller's (reused) buffer, as the bench's stream leg does
        out = np.full(len(data) * 2 + 4096, 0xEE, np.uint8) if rank == 0 and world == 8 else None
        g = shard.gather_blocks(blobs, st, dst=0, out=out)
        if rank == 0:
            if out is not None:
                assert np.shares_memory(g[1], out)
            c = avr.assemble_container(data, *g)
            with open(os.path.join(outdir, "out.avrc"), "wb") as f:
                f.write(c)
        else:
            assert g is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("realshort.mp4", 2), ("cockatoo.mp4", 2), ("realshort.mp4", 8)])
def test_gloo_world2_sharded_assembly(name, world):
    """The gather's message sequence (size all_gather, then per rank one metadata and one byte
    send / receive, the receives posted at once and drained in rank order) at world 2 and at the
    node's 8 ranks (there into a caller's buffer)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_gloo_worker, args=(world, port, name, td), nprocs=world, join=True)
        c = open(os.path.join(td, "out.avrc"), "rb").read()
    assert hashlib.sha256(c).hexdigest() == GOLD[(name, "P")]["avrc_sha256"]


# ------------------------------------------------------------- sharded decompress (host side)
def _container_payloads(data: bytes, avrc: bytes) -> list[bytes]:
    """The original payload bytes of each cabac block of a container, in block order (a coded
    block stands for `size` verbatim bytes of the file, recode.cpp:1275-1297)."""
    desc, _ = avr.describe_container(avrc)
    pos, out = 0, []
    for b in desc["blocks"]:
        if "literal" in b:
            pos += len(bytes.fromhex(b["literal"]))
        elif "cabac" in b:
            out.append(data[pos:pos + b["size"]])
            pos += b["size"]
    return out


def _oracle_p_container(name):
    from _oracle import oracle_cli
    return oracle_cli("compress", FIX / name, mode="P")


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_plan_and_splice_restore_the_file(name):
    """avr_plan_decompress lists the coded slices with their re-coded streams; avr_splice_container,
    fed each slice's payload, rebuilds the file (literals + slices + last-byte patch)."""
    data = (FIX / name).read_bytes()
    avrc = _oracle_p_container(name)
    plan = avr.plan_decompress(avrc)
    desc, _ = avr.describe_container(avrc)
    cabac = [bytes.fromhex(b["cabac"]) for b in desc["blocks"] if "cabac" in b]
    assert len(plan.descs) == len(cabac) > 0
    for d, c in zip(plan.descs, cabac):
        o, n = int(d["payload_offset"]), int(d["payload_size"])
        assert plan.arena[o:o + n].tobytes() == c
        assert int(d["out_offset"]) + int(d["out_capacity"]) <= plan.work_len
    pays = _container_payloads(data, avrc)
    lens = np.array([len(p) for p in pays], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    st = np.zeros(len(pays), np.int32)
    assert avr.splice_container(avrc, st, b"".join(pays), offs, lens) == data
    # a payload one byte short of its parity gets the stored last byte appended (recode.cpp:1349-1351)
    short = [p[:-1] for p in pays]
    lens2 = np.array([len(p) for p in short], np.uint32)
    offs2 = np.concatenate([[0], np.cumsum(lens2)[:-1]]).astype(np.uint64)
    assert avr.splice_container(avrc, st, b"".join(short), offs2, lens2) == data
    # a slice's bytes past the end of the gathered buffer are refused, not read
    with pytest.raises(avr.AvrError):
        avr.splice_container(avrc, st, b"".join(pays)[:-1], offs, lens)
    st[len(st) // 2] = -9
    with pytest.raises(avr.AvrError):
        avr.splice_container(avrc, st, b"".join(pays), offs, lens)


def test_plan_decompress_refuses_reference_model():
    from _oracle import oracle_cli
    avrc = oracle_cli("compress", FIX / "realshort.mp4", mode="R")
    with pytest.raises(avr.AvrError) as e:
        avr.plan_decompress(avrc)
    assert e.value.code == -6


def _gloo_decompress_worker(rank, world, port, name, outdir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = (FIX / name).read_bytes()
        avrc = _oracle_p_container(name)
        pays = _container_payloads(data, avrc)
        plan = avr.plan_decompress(avrc)
        lo, hi = shard.partition(plan.descs["payload_size"], world)[rank]

        def run_range(part):   # stands in for this rank's device decompress
            assert len(part.descs) == hi - lo
            mine = pays[lo:hi]
            lens = np.array([len(p) for p in mine], np.int64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            flat = torch.from_numpy(np.frombuffer(b"".join(mine) + b"\0" * 16, np.uint8).copy())
            return flat, np.zeros(len(mine), np.int64), offs, lens

        out = shard.sharded_decompress(None, avrc, run_range=run_range)
        if rank == 0:
            with open(os.path.join(outdir, "out.bin"), "wb") as f:
                f.write(out)
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_sharded_decompress_reassembles(world):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_gloo_decompress_worker, args=(world, port, "cockatoo.mp4", td), nprocs=world, join=True)
        out = open(os.path.join(td, "out.bin"), "rb").read()
    assert out == (FIX / "cockatoo.mp4").read_bytes()


def test_deal_files_lpt():
    rng = np.random.default_rng(3)
    sizes = rng.integers(1, 10_000_000, size=37)
    for world in (1, 2, 3, 8):
        owned = shard.deal_files(sizes, world)
        assert sorted(i for o in owned for i in o) == list(range(len(sizes)))
        loads = [int(sum(sizes[i] for i in o)) for o in owned]
        assert max(loads) <= sizes.sum() / world + sizes.max()
    assert shard.deal_files([], 4) == [[], [], [], []]
    assert shard.deal_files([5, 1, 1, 1, 1, 1], 2) == [[0], [1, 2, 3, 4, 5]]


def test_take_copies_buffers_past_2gib():
    """Library outputs of 2 GiB and more (a full-size configs[3] stream and its container) come back
    whole: ctypes.string_at's int length would wrap them (a 4.47 GB stream came back as 172 MB)."""
    import ctypes

    import avrecode_amd as avr
    libc = ctypes.CDLL(None)
    libc.malloc.restype = ctypes.c_void_p
    libc.malloc.argtypes = [ctypes.c_size_t]
    n = (1 << 31) + 4099
    p = libc.malloc(n)
    assert p
    ctypes.memset(p, 0x5A, n)
    ctypes.memset(p + n - 7, 0x33, 7)
    b = avr._take(ctypes.c_void_p(p), n)   # frees p
    assert len(b) == n and b[:4] == b"ZZZZ" and b[-8:] == b"Z" + b"\x33" * 7


def test_file_batch_calls_reject_bad_arguments_without_a_device():
    """avr_compress_files / avr_decompress_files / avr_roundtrip_files check their arguments
    before touching a context: a NULL context, a negative count or a NULL input is
    AVR_ERR_INVALID_ARGUMENT (-1), on any host."""
    import ctypes
    L = avr.lib()
    buf = ctypes.create_string_buffer(b"x" * 16)
    ins = (ctypes.c_void_p * 1)(ctypes.cast(buf, ctypes.c_void_p).value)
    lens = (ctypes.c_size_t * 1)(16)
    outs = (ctypes.c_void_p * 1)()
    olens = (ctypes.c_size_t * 1)()
    st = (ctypes.c_int32 * 1)()
    times = (ctypes.c_double * 2)()
    assert L.avr_roundtrip_files(None, 1, ins, lens, avr.MODEL_PARALLEL, outs, olens, st, times) == -1
    assert L.avr_compress_files(None, 1, ins, lens, avr.MODEL_PARALLEL, outs, olens, st) == -1
    assert L.avr_decompress_files(None, 1, ins, lens, outs, olens, st) == -1
    fake = ctypes.c_void_p(1)   # never dereferenced: the argument checks fail first
    assert L.avr_roundtrip_files(fake, -1, ins, lens, avr.MODEL_PARALLEL, outs, olens, st, times) == -1
    assert L.avr_roundtrip_files(fake, 1, ins, lens, 7, outs, olens, st, times) == -1
    assert L.avr_roundtrip_files(fake, 1, ins, lens, avr.MODEL_PARALLEL, outs, olens, None, times) == -1
    nul = (ctypes.c_void_p * 1)()
    assert L.avr_roundtrip_files(fake, 1, nul, lens, avr.MODEL_PARALLEL, outs, olens, st, times) == -1
