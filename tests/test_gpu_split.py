"""The parallel model's long-slice split on the device (avr_k_split.hip; include/avrecode.h
avr_set_split_bytes; the format restated by the oracle, oracle/oracle_seams.c).

* x264 fixtures at small split sizes: the device's containers equal the oracle's byte for byte
  (pieces' streams, seams fields: cut positions, re-encoder states, context states, upper-row edges),
  through the checked single-file compress and the batched one, and decompress on the device (one
  workgroup per piece) to the input;
* a 4K 4:4:4 intra slice (the configs[4] corpus's floor) at the default split size: cut into pieces,
  equal to the oracle's container, restored by the device, and the oracle's sequential decompress of
  the device's container restores it too;
* split off (0): no seams, the plain parallel-model container."""
import tempfile
from pathlib import Path

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


def _cut_blocks(avrc):
    info, _ = avr.describe_container(avrc)
    return [b for b in info["blocks"] if "seams" in b]


@pytest.mark.parametrize("split_bytes", [512, 2048])
@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_fixture_split_matches_oracle(ctx, name, split_bytes):
    data = (FIX / name).read_bytes()
    ctx.split_bytes = split_bytes
    try:
        avrc = ctx.compress(data, avr.MODEL_PARALLEL)          # checked: pieces decompressed and compared
        assert _cut_blocks(avrc)
        assert avrc == oracle_cli("compress", FIX / name, mode="P", split_bytes=split_bytes)
        assert ctx.decompress(avrc) == data
        outs = ctx.compress_files([data, data], avr.MODEL_PARALLEL)
        assert outs == [avrc, avrc]
        back, _ = ctx.roundtrip_files([data], avr.MODEL_PARALLEL)   # unchecked first pass
        assert back == [avrc]
    finally:
        ctx.split_bytes = avr.SPLIT_BYTES_DEFAULT


def test_split_off_is_the_plain_container(ctx):
    data = (FIX / "realshort.mp4").read_bytes()
    ctx.split_bytes = 0
    try:
        avrc = ctx.compress(data, avr.MODEL_PARALLEL)
        assert not _cut_blocks(avrc)
        assert avrc == oracle_cli("compress", FIX / "realshort.mp4", mode="P", split_bytes=0)
    finally:
        ctx.split_bytes = avr.SPLIT_BYTES_DEFAULT


def test_4k_444_intra_slice_is_split(ctx):
    data = ctx.synthesize(avr.SynthParams(mb_width=240, mb_height=135, slice_type=2, slice_qp=30, chroma_format_idc=3,
                                          transform_8x8_mode=1, seed=4006, slices_per_picture=1, gop_length=1), 1)
    assert ctx.split_bytes == avr.SPLIT_BYTES_DEFAULT
    avrc = ctx.compress(data, avr.MODEL_PARALLEL)
    cut = _cut_blocks(avrc)
    assert len(cut) == 1
    assert ctx.decompress(avrc) == data
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "k.264"
        f.write_bytes(data)
        assert avrc == oracle_cli("compress", f, mode="P", split_bytes=avr.SPLIT_BYTES_DEFAULT)
        g = Path(td) / "k.avrc"
        g.write_bytes(avrc)
        assert oracle_cli("decompress", g) == data



def test_synthetic_corpus_split_matches_oracle(ctx):
    """Cuts in every slice kind the generator makes: P and B slices (mvd, ref_idx and direct flags in
    the upper-row edges), 4:2:0 / 4:2:2 / 4:4:4, 8x8 transforms, several slices per
    picture (slices that start mid-row: the edges of the columns before the start are empty), and
    field / MBAFF streams, which are never cut."""
    specs = [(22, 18, 2, 6, 6, 1, 25, 1, 0), (14, 9, 3, 5, 5, 0, 27, 3, 0), (30, 17, 1, 4, 2, 2, 29, 2, 0),
             (11, 7, 1, 7, 4, 1, 23, 1, 0), (40, 23, 3, 4, 4, 1, 24, 1, 0), (20, 12, 1, 4, 4, 0, 26, 1, 1),
             (20, 12, 1, 4, 4, 1, 26, 1, 2)]
    ctx.split_bytes = 700
    try:
        with tempfile.TemporaryDirectory() as td:
            datas = []
            for k, (w, h, spf, frames, gop, st, qp, cf, structure) in enumerate(specs):
                p = avr.SynthParams(mb_width=w, mb_height=h, slice_type=st, slice_qp=qp, chroma_format_idc=cf,
                                    seed=900 + k, slices_per_picture=spf, gop_length=gop, num_ref_idx_l0=2,
                                    structure=structure)
                data = ctx.synthesize(p, frames)
                datas.append(data)
                f = Path(td) / f"s{k}.264"
                f.write_bytes(data)
                avrc = ctx.compress(data, avr.MODEL_PARALLEL)
                assert avrc == oracle_cli("compress", f, mode="P", split_bytes=700), k
                assert bool(avr.seams_of_container(avrc)) == (structure == 0), k
            outs = ctx.compress_files(datas, avr.MODEL_PARALLEL)
            assert ctx.decompress_files(outs) == datas
    finally:
        ctx.split_bytes = avr.SPLIT_BYTES_DEFAULT


def test_hooks_decompress_reads_a_split_container(ctx):
    """The libavcodec-hooks decompress session over a split container: the callbacks of every
    slice are served (the driver's parse walks them all) and avr_hooks_end returns the file."""
    from test_hooks import _call
    data = (FIX / "cockatoo.mp4").read_bytes()
    ctx.split_bytes = 1024
    try:
        avrc = ctx.compress(data, avr.MODEL_PARALLEL)
    finally:
        ctx.split_bytes = avr.SPLIT_BYTES_DEFAULT
    assert avr.seams_of_container(avrc)
    r, back, walked = _call("hooks_decompress", avrc, len(avrc))
    assert r == 0, r
    assert back == data and walked > 0


def test_damaged_seams_are_refused(ctx):
    """A seams field that does not parse or describes impossible cuts fails the file with
    AVR_ERR_FORMAT (-3) instead of launching pieces from it; a damaged piece stream fails too."""
    data = (FIX / "realshort.mp4").read_bytes()
    ctx.split_bytes = 1024
    try:
        avrc = ctx.compress(data, avr.MODEL_PARALLEL)
    finally:
        ctx.split_bytes = avr.SPLIT_BYTES_DEFAULT
    info, _ = avr.describe_container(avrc)
    blob = bytes.fromhex(next(b["seams"] for b in info["blocks"] if "seams" in b))
    i = avrc.index(blob)
    bad = bytearray(avrc)
    bad[i + len(blob) // 2] ^= 0x55          # inside the zlib stream
    back = ctx.decompress_files([bytes(bad), avrc])
    assert isinstance(back[0], avr.AvrError) and back[0].code == -3
    assert back[1] == data                   # the batch's other file is unaffected
