"""Several files at once (avr_compress_files / avr_decompress_files): the reference model's unit of
sequential work is a file (its estimators persist across ITS slices, recode.cpp:662-665), so a
corpus runs its files side by side.  Every file's container must equal the single-file call's and
the oracle's (.avrc bytes), in both model modes, and decompress must restore every file; a bad file
fails alone.  Also the configs[4] corpus generator (avrecode_amd/workloads.py) and the configs[3]
tiled stream, at small sizes."""
import hashlib
import json
import tempfile
from pathlib import Path

import pytest

from _oracle import ROOT, oracle_cli

torch = pytest.importorskip("torch")
import avrecode_amd as avr  # noqa: E402
from avrecode_amd import workloads  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}
MODELS = (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL))


@pytest.fixture(scope="module")
def ctx():
    c = avr.Context(0)
    yield c
    c.close()


def _small_corpus(ctx):
    files = []
    specs = [(22, 18, 2, 6, 6, 1, 25, 1), (14, 9, 3, 5, 5, 0, 27, 3), (30, 17, 1, 4, 2, 2, 29, 2),
             (11, 7, 1, 7, 4, 1, 23, 1)]
    for k, (w, h, spf, frames, gop, st, qp, cf) in enumerate(specs):
        p = avr.SynthParams(mb_width=w, mb_height=h, slice_type=st, slice_qp=qp, chroma_format_idc=cf, seed=300 + k,
                            slices_per_picture=spf, gop_length=gop, num_ref_idx_l0=2)
        files.append((f"s{k}", ctx.synthesize(p, frames)))
    for f in workloads.FIXTURES:
        files.append((f, (ROOT / "tests" / "fixtures" / f).read_bytes()))
    return files


def test_small_corpus_matches_oracle_and_single_file(ctx):
    files = _small_corpus(ctx)
    datas = [d for _, d in files]
    with tempfile.TemporaryDirectory() as td:
        for mode, model in MODELS:
            outs = ctx.compress_files(datas, model)
            for (name, data), avrc in zip(files, outs):
                assert isinstance(avrc, bytes), (name, avrc)
                assert avrc == ctx.compress(data, model), (name, mode)
                if (name, mode) in GOLD:
                    assert hashlib.sha256(avrc).hexdigest() == GOLD[(name, mode)]["avrc_sha256"]
                else:
                    f = Path(td) / f"{name}.264"
                    f.write_bytes(data)
                    assert avrc == oracle_cli("compress", f, mode=mode), (name, mode)
            back = ctx.decompress_files(outs)
            assert back == datas, mode


def test_mixed_models_and_error_isolation(ctx):
    files = _small_corpus(ctx)
    datas = [d for _, d in files]
    r = ctx.compress_files(datas, avr.MODEL_REFERENCE)
    p = ctx.compress_files(datas, avr.MODEL_PARALLEL)
    mixed = [r[k] if k % 2 else p[k] for k in range(len(datas))]
    bad = bytearray(mixed[1])
    bad[len(bad) // 2] ^= 0x5A
    batch = mixed + [bytes(bad), b"\x12\x05\x08"]
    back = ctx.decompress_files(batch)
    assert back[:len(datas)] == datas
    assert isinstance(back[-1], avr.AvrError)
    # a corrupted container either fails or (if the flip hit a literal) decodes to something else
    assert isinstance(back[-2], avr.AvrError) or back[-2] != datas[1]
    outs = ctx.compress_files([datas[0], b"not h264 at all", datas[2]], avr.MODEL_REFERENCE)
    assert outs[0] == r[0] and outs[2] == r[2] and isinstance(outs[1], avr.AvrError)


@pytest.mark.parametrize("force_verify", [False, True])
@pytest.mark.parametrize("mode,model", MODELS + (("P32", avr.MODEL_PARALLEL32),))
def test_roundtrip_files(ctx, monkeypatch, mode, model, force_verify):
    """avr_roundtrip_files: the unchecked first pass (or, forced, the checked second one) gives
    every file the container avr_compress_files gives it, and a file that cannot be compressed
    fails alone."""
    if force_verify:
        monkeypatch.setenv("AVR_ROUNDTRIP_FORCE_VERIFY", "1")
    files = _small_corpus(ctx)
    datas = [d for _, d in files]
    want = ctx.compress_files(datas, model)
    outs, times = ctx.roundtrip_files(datas + [b"not h264 at all"], model)
    assert outs[:-1] == want, mode
    assert isinstance(outs[-1], avr.AvrError)
    assert times["compress_s"] > 0 and times["decompress_s"] > 0
    assert ctx.decompress_files(outs[:-1]) == datas


def test_corpus_generator_structure(ctx):
    files = workloads.corpus(ctx, scale=0.25, fixtures=False)
    assert [n for n, _ in files] == [c[0] for c in workloads.CORPUS]
    for entry, (_, data) in zip(workloads.CORPUS, files):
        name, w, h, spf, frames, gop, st, qp, cf, structure = entry
        d = avr.parse_stream(data).descs
        n = max(1, int(round(frames * 0.25)))
        assert len(d) == workloads.slices_of(entry, n), name
        assert (d["mb_width"] == w).all() and (d["mb_height"] == h).all() and (d["chroma_array_type"] == cf).all()
        want = {0: {0}, 1: {1, 2}, 2: {3}}[structure]
        assert set(int(x) for x in d["structure"]) == want, name
        types = set(int(t) for t in d["slice_type"])
        assert 2 in types
    outs = ctx.compress_files([d for _, d in files], avr.MODEL_REFERENCE)
    assert ctx.decompress_files(outs) == [d for _, d in files]


def test_tiled_stream_small(ctx):
    data = workloads.stream_4k(ctx, seconds=3, fps=5, mb_width=20, mb_height=12)
    d = avr.parse_stream(data).descs
    assert len(d) == 15
    assert [int(t) for t in d["slice_type"]] == [2, 0, 0, 0, 0] * 3
    assert len(set(int(x) for x in d["picture_id"])) == 15
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "t.264"
        f.write_bytes(data)
        for mode, model in MODELS:
            avrc = ctx.compress(data, model)
            assert avrc == oracle_cli("compress", f, mode=mode), mode
            assert ctx.decompress(avrc) == data
