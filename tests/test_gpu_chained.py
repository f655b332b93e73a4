"""The chained reference model (AVR_MODEL_CHAINED, "avrecode-amd:R16"): the reference model with a
fresh model before every 16th coded slice of a file.  Its containers must equal the oracle's
(tests/test_oracle_fixtures.py pins each chain to the reference model run on that chain alone), on
every device path the reference model has -- the parallel R-mode compress pass with chains as its
files, the per-chain sequential kernel, batches of several files -- and its decompress runs one
workgroup per chain.
"""
import time

import pytest

from _oracle import ROOT, oracle_cli

torch = pytest.importorskip("torch")
import avrecode_amd as avr  # noqa: E402

pytestmark = pytest.mark.gpu
FIX = ROOT / "tests" / "fixtures"


@pytest.fixture(scope="module")
def ctx():
    c = avr.Context(0)
    yield c
    c.close()


def _tiled(copies=5, lead=0):
    """The PAFF fixture's 8 slices tiled; lead > 0 repeats the first GOP's first `lead` slices before
    the tiles, so that chain boundaries fall on P fields inside a GOP."""
    import bench
    head, sl = bench._split_slices((FIX / "paff_ipp.264").read_bytes())
    return head + b"".join(sl[:lead] + sl * copies)


def _oracle_c(data, tmp_path, name="x.264"):
    f = tmp_path / name
    f.write_bytes(data)
    return oracle_cli("compress", f, mode="C")


@pytest.mark.parametrize("lead", [0, 3], ids=["idr_aligned", "mid_gop"])
def test_chained_every_compress_path_matches_oracle(ctx, tmp_path, monkeypatch, lead):
    """40 (43) field slices, three chains: whichever path the cost rule picks, the parallel R-mode
    pass with chains as files (AVR_RMODE_PARALLEL) and one sequential workgroup per chain
    (AVR_RMODE_SEQUENTIAL) give the oracle's container, and it decompresses back."""
    data = _tiled(lead=lead)
    ref = _oracle_c(data, tmp_path)
    assert avr.container_model(ref) == avr.MODEL_CHAINED
    assert ctx.compress(data, avr.MODEL_CHAINED) == ref
    monkeypatch.setenv("AVR_RMODE_PARALLEL", "1")
    assert ctx.compress(data, avr.MODEL_CHAINED) == ref
    monkeypatch.delenv("AVR_RMODE_PARALLEL")
    monkeypatch.setenv("AVR_RMODE_SEQUENTIAL", "1")
    assert ctx.compress(data, avr.MODEL_CHAINED) == ref
    monkeypatch.delenv("AVR_RMODE_SEQUENTIAL")
    assert ctx.decompress(ref) == data
    assert ctx.decompress(oracle_cli("compress", tmp_path / "x.264", mode="R")) == data   # R unchanged


def test_chained_file_batch(ctx, tmp_path):
    """Several files in one batch, chains of each file cut independently: every container equals
    the oracle's for that file alone, and the batched decompress restores every file."""
    datas = [_tiled(3), (FIX / "cockatoo.mp4").read_bytes(), (FIX / "realshort.mp4").read_bytes(), _tiled(2)]
    outs = ctx.compress_files(datas, avr.MODEL_CHAINED)
    for i, (d, o) in enumerate(zip(datas, outs)):
        assert o == _oracle_c(d, tmp_path, f"f{i}.bin"), i
    assert ctx.decompress_files(outs) == datas


def test_chained_roundtrip_and_ratio(ctx):
    """avr_roundtrip_file in the chained model; its container sits between the reference model's
    and the parallel model's (realshort: R 0.990, C 0.998, P 1.041)."""
    data = (FIX / "realshort.mp4").read_bytes()
    c, st = ctx.roundtrip(data, avr.MODEL_CHAINED)
    r = ctx.compress(data, avr.MODEL_REFERENCE)
    p = ctx.compress(data, avr.MODEL_PARALLEL)
    assert len(r) <= len(c) < len(p) and len(c) < len(data)


def test_chained_decompress_runs_chains_at_once(ctx):
    """cockatoo.mp4 (267 coded slices: 17 chains): the chained container decompresses on one
    workgroup per chain, several times faster than the reference model's one chain (3.6 s)."""
    data = (FIX / "cockatoo.mp4").read_bytes()
    r = ctx.compress(data, avr.MODEL_REFERENCE)
    c = ctx.compress(data, avr.MODEL_CHAINED)
    ctx.decompress(c)   # warm
    t0 = time.perf_counter()
    assert ctx.decompress(r) == data
    t_r = time.perf_counter() - t0
    t0 = time.perf_counter()
    assert ctx.decompress(c) == data
    t_c = time.perf_counter() - t0
    print(f"cockatoo decompress: R {t_r:.3f} s, chained {t_c:.3f} s")
    assert t_c < 0.5 * t_r


def test_chained_refused_by_slice_batches(ctx):
    """A slice batch has no file to chain over: it refuses the chained model (whole-file calls, the
    hooks sessions -- streaming ones too, since round 6: tests/test_hooks.py -- and the per-rank chain
    ranges take it)."""
    z = torch.zeros(16, dtype=torch.uint8, device="cuda")
    with pytest.raises(avr.AvrError):
        ctx.compress_slices(z, 0, 1, 1, z, z, z, model=avr.MODEL_CHAINED)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_chain_ranges_in_one_process_equal_whole_file(ctx, world):
    """Every rank's chain range run in this process (avr_compress_chain_range /
    avr_decompress_chain_range), concatenated in rank order, assembles / splices to exactly the
    whole-file container and file: the chained model sharded within a file."""
    import numpy as np
    data = _tiled(copies=6, lead=3)   # 51 slices: 4 chains
    whole = ctx.compress(data, avr.MODEL_CHAINED)
    parts = [ctx.compress_chain_range(data, world, r) for r in range(world)]
    assert parts[0][0] == 0 and all(parts[r][1] == parts[r + 1][0] for r in range(world - 1))
    st = np.concatenate([p[2] for p in parts])
    assert len(st) == parts[-1][1] and not (st < -1).any()
    if world > 1:
        assert sum(p[1] > p[0] for p in parts) > 1, "the chains should spread over the ranks"
    blob, offs, base = [], [], 0
    for p in parts:
        blob.append(p[3])
        offs.append(p[4].astype(np.uint64) + base)
        base += len(p[3])
    avrc = avr.assemble_container(data, st, np.concatenate(blob), np.concatenate(offs),
                                  np.concatenate([p[5] for p in parts]), model=avr.MODEL_CHAINED)
    assert avrc == whole
    dparts = [ctx.decompress_chain_range(whole, world, r) for r in range(world)]
    dst = np.concatenate([p[2] for p in dparts])
    dblob, doffs, base = [], [], 0
    for p in dparts:
        dblob.append(p[3])
        doffs.append(p[4].astype(np.uint64) + base)
        base += len(p[3])
    out = avr.DecompressPlan().load(whole).splice(dst, np.concatenate(dblob), np.concatenate(doffs),
                                                  np.concatenate([p[5] for p in dparts]))
    assert out.tobytes() == data


@pytest.mark.parametrize("name,world", [("cockatoo.mp4", 2), ("cockatoo.mp4", 3), ("realshort.mp4", 2)])
def test_sharded_chained_multirank_gloo(name, world, tmp_path):
    """The chained model across ranks in separate processes (all on cuda:0, gloo for the gathers):
    shard.sharded_compress_chained equals the single-GPU container (and the oracle's), and
    shard.sharded_decompress_chained restores the file."""
    import os
    import socket
    import subprocess
    import sys
    from pathlib import Path
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "out.avrc"
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).parent / "_shard_worker.py"),
                                       str(FIX / name), str(out), "C"], env=env))
    rcs = [p.wait(timeout=110) for p in procs]
    assert rcs == [0] * world, rcs
    assert out.read_bytes() == oracle_cli("compress", FIX / name, mode="C")
    assert Path(str(out) + ".dec").read_bytes() == (FIX / name).read_bytes()
