"""The north-star command itself on the device: `recode compress|decompress|roundtrip [-p]`
(avrecode_amd/recode, mirroring main/roundtrip, recode.cpp:1594-1659), run as a subprocess on both
fixtures in both model modes.  The .avrc bytes must equal the committed goldens (the oracle's
output, tests/golden/fixtures.json), decompress must restore the input, and the protobuf runtime
must parse the container (recode.proto).  Also the sharded compress (avrecode_amd/shard.py) at
world size 1 over RCCL, byte-identical to the single-GPU compress."""
import hashlib
import json
import os
import socket
import subprocess
import tempfile
from pathlib import Path

import pytest

import _pb
from _oracle import ROOT

pytestmark = pytest.mark.gpu
FIX = ROOT / "tests" / "fixtures"
CLI = ROOT / "avrecode_amd" / "recode"
GOLD = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}
CASES = [(f, m) for f in ("realshort.mp4", "cockatoo.mp4") for m in ("R", "P", "C")]
FLAGS = {"R": [], "P": ["-p"], "C": ["-c"]}


def _run(args, timeout=120):
    assert CLI.exists(), "recode CLI not built (make -C avrecode_amd)"
    return subprocess.run([str(CLI)] + [str(a) for a in args], capture_output=True, timeout=timeout)


@pytest.mark.parametrize("name,mode", CASES)
def test_cli_roundtrip(name, mode):
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "x.avrc"
        args = ["roundtrip"] + FLAGS[mode] + [FIX / name, out]
        r = _run(args)
        assert r.returncode == 0, r.stderr.decode()
        text = r.stdout.decode()
        assert "Compress-decompress roundtrip succeeded" in text
        avrc = out.read_bytes()
    g = GOLD[(name, mode)]
    assert len(avrc) == g["avrc_len"]
    assert hashlib.sha256(avrc).hexdigest() == g["avrc_sha256"]


@pytest.mark.parametrize("name,mode", CASES)
def test_cli_compress_then_decompress(name, mode):
    data = (FIX / name).read_bytes()
    with tempfile.TemporaryDirectory() as td:
        c, d = Path(td) / "c.avrc", Path(td) / "d.mp4"
        r = _run(["compress"] + FLAGS[mode] + [FIX / name, c])
        assert r.returncode == 0, r.stderr.decode()
        avrc = c.read_bytes()
        assert hashlib.sha256(avrc).hexdigest() == GOLD[(name, mode)]["avrc_sha256"]
        m = _pb.check_container(avrc, data)
        assert bool(m.HasField("metadata")) == (mode != "R")
        r = _run(["decompress", c, d])
        assert r.returncode == 0, r.stderr.decode()
        assert d.read_bytes() == data


def test_cli_errors():
    with tempfile.TemporaryDirectory() as td:
        bad = Path(td) / "bad.avrc"
        bad.write_bytes(b"\x12\x05\x08")
        assert _run(["decompress", bad, Path(td) / "o"]).returncode != 0
        assert _run(["roundtrip", Path(td) / "missing.mp4"]).returncode != 0
        assert _run(["frobnicate", FIX / "realshort.mp4"]).returncode != 0


def test_sharded_compress_world1_rccl():
    import torch
    import torch.distributed as dist

    import avrecode_amd as avr
    from avrecode_amd import shard

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        with avr.Context(0) as ctx:
            for name in ("realshort.mp4", "cockatoo.mp4"):
                data = (FIX / name).read_bytes()
                got = shard.sharded_compress(ctx, data)
                assert got == ctx.compress(data, avr.MODEL_PARALLEL)
                assert hashlib.sha256(got).hexdigest() == GOLD[(name, "P")]["avrc_sha256"]
                # and back: the container's slices regenerated, gathered over RCCL, spliced on rank 0
                assert shard.sharded_decompress(ctx, got) == data
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_compress_multirank_gloo(world):
    """The sharded compress and decompress with several ranks, each a process of its own running its slice range
    on the device (all on cuda:0 here; one per GPU on a node), gathered to rank 0 over gloo: the
    container equals the single-GPU compress (golden sha) for both fixtures."""
    import subprocess
    import sys
    import tempfile

    for name in ("realshort.mp4", "cockatoo.mp4"):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        with tempfile.TemporaryDirectory() as td:
            out = Path(td) / "out.avrc"
            procs = []
            for r in range(world):
                env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                           WORLD_SIZE=str(world), LOCAL_RANK="0")
                procs.append(subprocess.Popen([sys.executable, str(Path(__file__).parent / "_shard_worker.py"),
                                               str(FIX / name), str(out)], env=env))
            rcs = [p.wait(timeout=100) for p in procs]
            assert rcs == [0] * world, rcs
            got = out.read_bytes()
            assert hashlib.sha256(got).hexdigest() == GOLD[(name, "P")]["avrc_sha256"], name
            # the worker also decompressed that container across the ranks (sharded_decompress)
            assert Path(str(out) + ".dec").read_bytes() == (FIX / name).read_bytes(), name


def _bills(stderr: str) -> dict:
    """The "Avrecode Bill" / "CABAC Bill" sections of ~h264_model's stderr print (recode.cpp:634-655)."""
    out, cur = {}, None
    for line in stderr.splitlines():
        if line in ("Avrecode Bill", "CABAC Bill"):
            cur = out.setdefault(line, {})
        elif " : " in line and cur is not None:
            k, v = line.split(" : ")
            cur[k.strip()] = int(v)
    return out


@pytest.mark.parametrize("name,mode", CASES)
def test_cli_billing_matches_oracle(name, mode):
    """h264_model::bill (re-coded bytes per put by CodingType, compress) and cabac_bill (CABAC bytes
    per put, decompress) -- recode.cpp:615-661, 1074-1078, 1213-1220, 1443-1468 -- equal the oracle's."""
    from _oracle import build_oracle
    _, oracle = build_oracle()
    args = ["roundtrip"] + FLAGS[mode] + [str(FIX / name)]
    r = _run(args)
    assert r.returncode == 0, r.stderr.decode()
    o = subprocess.run([str(oracle)] + args, capture_output=True, timeout=300)
    assert o.returncode == 0
    got, want = _bills(r.stderr.decode()), _bills(o.stderr.decode())
    assert want["Avrecode Bill"] and want["CABAC Bill"]
    assert got == want
    # the bills account for every re-coded byte but the finish() flushes (one per coded slice at most
    # a handful of bytes), and for every regenerated CABAC byte likewise
    data = (FIX / name).read_bytes()
    import avrecode_amd as avr
    with avr.Context(0) as ctx:
        _, st = ctx.roundtrip(data, {"R": avr.MODEL_REFERENCE, "P": avr.MODEL_PARALLEL, "C": avr.MODEL_CHAINED}[mode])
    assert st["bill"] == want["Avrecode Bill"] and st["cabac_bill"] == want["CABAC Bill"]
    assert 0 <= st["recoded_bytes"] - sum(st["bill"].values()) <= 16 * st["coded_slices"]
