"""Field-coded H.264: field pictures (PAFF) and MBAFF frames, from the device
generator (avr_synthesize_stream, structure 1 / 2), against the oracle.

What the fork does for these (FFmpeg h264_cabac.c / h264_slice.c, restated in oracle_walker.c):
field-coded macroblocks take the field ctxIdx offsets of significant / last_significant_coeff_flag
and the field 8x8 significance map (recode.cpp:691-694 holds that map); the model keys of those
bins do not change (recode.cpp:686-704 uses the frame map and frame offsets), the model hooks see
FFmpeg's frame row of each macroblock (a field picture's row r is frame row 2 r + bottom) and the
frame's size, and the two fields of a frame share frame_num, so frame_spec keeps one model frame
for both.  No interlaced stream of the reference or of a real encoder is present:
parity here is product against oracle, both restating the published algorithm."""
import os
import tempfile
from pathlib import Path

import pytest

from _oracle import oracle_cli

torch = pytest.importorskip("torch")
import avrecode_amd as avr  # noqa: E402
from test_gpu_parity import _check_batch_against_oracle  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = avr.Context(0)
    yield c
    c.close()


def _paff(ctx, n, **kw):
    args = dict(mb_width=14, mb_height=10, slice_type=0, slice_qp=26, seed=5, structure=1)
    args.update(kw)
    return ctx.synthesize(avr.SynthParams(**args), n)


def test_field_pictures_structure(ctx):
    data = _paff(ctx, 4, gop_length=2, slices_per_picture=2)
    d = avr.parse_stream(data).descs
    assert len(d) == 4 * 2 * 2
    assert [int(x) for x in d["structure"]] == [1, 1, 2, 2] * 4
    # the two fields of a frame share the model's frame (frame_num), frames advance
    assert [int(x) for x in d["picture_id"]] == [k // 4 + 1 for k in range(16)]
    assert (d["mb_height"] == 10).all() and [int(x) for x in d["first_mb"]] == [0, 35] * 8
    assert [int(t) for t in d["slice_type"]] == [2] * 4 + [0] * 4 + [2] * 4 + [0] * 4


CASES = [
    # (slice_type, chroma, t8, l0, l1, gop, spp)
    (2, 1, 1, 1, 1, 0, 1),
    (0, 1, 1, 2, 1, 3, 1),
    (1, 1, 1, 2, 2, 4, 2),
    (0, 2, 1, 1, 1, 2, 1),
    (1, 3, 1, 1, 3, 3, 1),
    (0, 3, 0, 3, 1, 0, 3),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_field_picture_slices_match_oracle(ctx, case):
    st, cf, t8, l0, l1, gop, spp = case
    data = _paff(ctx, 3, slice_type=st, chroma_format_idc=cf, transform_8x8_mode=t8, num_ref_idx_l0=l0,
                 num_ref_idx_l1=l1, gop_length=gop, slices_per_picture=spp, seed=40 + st + 3 * cf)
    ps, verdict = _check_batch_against_oracle(ctx, data, require_all=True)
    assert len(ps.descs) == 3 * 2 * spp


@pytest.mark.parametrize("case", CASES[1:5], ids=lambda c: "x".join(map(str, c)))
def test_field_picture_files_match_oracle(ctx, case, monkeypatch):
    """Whole files in both model modes: the reference model's frame-row coordinates, shared
    frame per field pair and previous-frame contexts, against the oracle; the parallel
    reference-model compress against the sequential kernel."""
    monkeypatch.setenv("AVR_RMODE_PARALLEL", "1")   # the parallel R-mode compress, whatever the cost rule picks
    st, cf, t8, l0, l1, gop, spp = case
    data = _paff(ctx, 4, slice_type=st, chroma_format_idc=cf, transform_8x8_mode=t8, num_ref_idx_l0=l0,
                 num_ref_idx_l1=l1, gop_length=gop, slices_per_picture=spp, seed=70 + st + 3 * cf)
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "paff.264"
        f.write_bytes(data)
        for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL)):
            avrc = ctx.compress(data, model)
            assert avrc == oracle_cli("compress", f, mode=mode), mode
            assert ctx.decompress(avrc) == data
    os.environ["AVR_RMODE_SEQUENTIAL"] = "1"
    try:
        seq = ctx.compress(data, avr.MODEL_REFERENCE)
    finally:
        del os.environ["AVR_RMODE_SEQUENTIAL"]
    assert seq == ctx.compress(data, avr.MODEL_REFERENCE)


def test_bottom_field_first(ctx, monkeypatch):
    """Field pictures with the bottom field coded first (generator structure 3): the bottom field
    is the IDR / first field, the top field the second field of the same frame_num, so the two
    still share one picture id; the reference model's first-coded field is the bottom one (its
    parallel compress must see the top rows as not yet written).  Batch, both file models, the
    sequential reference-model compress, against the oracle."""
    monkeypatch.setenv("AVR_RMODE_PARALLEL", "1")   # the parallel R-mode compress, whatever the cost rule picks
    data = _paff(ctx, 4, structure=3, slice_type=1, gop_length=3, slices_per_picture=2, num_ref_idx_l0=2,
                 transform_8x8_mode=1, seed=91)
    d = avr.parse_stream(data).descs
    assert [int(x) for x in d["structure"][:8]] == [2, 2, 1, 1] * 2
    assert [int(x) for x in d["picture_id"]] == [k // 4 + 1 for k in range(16)]
    _check_batch_against_oracle(ctx, data, require_all=True)
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "bff.264"
        f.write_bytes(data)
        for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL)):
            avrc = ctx.compress(data, model)
            assert avrc == oracle_cli("compress", f, mode=mode), mode
            assert ctx.decompress(avrc) == data
    os.environ["AVR_RMODE_SEQUENTIAL"] = "1"
    try:
        seq = ctx.compress(data, avr.MODEL_REFERENCE)
    finally:
        del os.environ["AVR_RMODE_SEQUENTIAL"]
    assert seq == ctx.compress(data, avr.MODEL_REFERENCE)


def test_field_and_frame_pictures_mixed(ctx):
    """A progressive stream followed by a field stream of the same size (two SPS): frame and field
    context tables alternate in one reference-model walk."""
    a = ctx.synthesize(avr.SynthParams(mb_width=12, mb_height=8, slice_type=0, slice_qp=27, seed=8), 2)
    b = _paff(ctx, 2, mb_width=12, mb_height=8, slice_type=0, seed=9, gop_length=2)
    data = a + b + a
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "mix.264"
        f.write_bytes(data)
        for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL)):
            avrc = ctx.compress(data, model)
            assert avrc == oracle_cli("compress", f, mode=mode), mode
            assert ctx.decompress(avrc) == data


@pytest.mark.parametrize("name", ["paff_ipp.264", "mbaff_ib.264"])
def test_field_fixture_matches_golden(ctx, name):
    """The committed field-coded streams (tests/golden/fields.json) compress to the oracle's
    pinned containers in both model modes and decompress back."""
    import hashlib
    import json
    g = {e["file"]: e for e in json.loads((Path(__file__).parent / "golden" / "fields.json").read_text())["files"]}[name]
    data = (Path(__file__).parent / "fixtures" / name).read_bytes()
    for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL), ("C", avr.MODEL_CHAINED)):
        avrc = ctx.compress(data, model)
        assert hashlib.sha256(avrc).hexdigest() == g[mode]["avrc_sha256"], mode
        assert ctx.decompress(avrc) == data


# ------------------------------------------------------------------------------ MBAFF frames
def _mbaff(ctx, n, **kw):
    args = dict(mb_width=11, mb_height=8, slice_type=0, slice_qp=27, seed=3, structure=2)
    args.update(kw)
    return ctx.synthesize(avr.SynthParams(**args), n)


def test_mbaff_structure(ctx):
    data = _mbaff(ctx, 3, gop_length=2, slices_per_picture=2)
    d = avr.parse_stream(data).descs
    assert len(d) == 3 * 2
    assert (d["structure"] == 3).all() and (d["mb_height"] == 8).all()
    # first_mb_in_slice counts pairs: 44 pairs split 22 / 22 -> macroblocks 0 and 44
    assert [int(x) for x in d["first_mb"]] == [0, 44] * 3
    assert [int(x) for x in d["picture_id"]] == [1, 1, 2, 2, 3, 3]


MBAFF_CASES = [
    # (slice_type, chroma, t8, l0, l1, gop, spp)
    (2, 1, 0, 1, 1, 0, 1),
    (2, 1, 1, 1, 1, 0, 1),
    (0, 1, 1, 2, 1, 3, 1),
    (1, 1, 1, 2, 2, 4, 1),
    (0, 2, 0, 1, 1, 2, 1),
    (1, 3, 1, 1, 2, 3, 1),
    (0, 1, 0, 1, 1, 2, 3),
]


@pytest.mark.parametrize("case", MBAFF_CASES, ids=lambda c: "x".join(map(str, c)))
def test_mbaff_slices_match_oracle(ctx, case):
    """Macroblock pairs (Table 6-4 neighbours, skip / field-flag order, field-pair context tables
    and doubled references) slice by slice: the device generator's stream parses in the oracle,
    and the device's re-coded / regenerated bytes equal the oracle's."""
    st, cf, t8, l0, l1, gop, spp = case
    data = _mbaff(ctx, 3, slice_type=st, chroma_format_idc=cf, transform_8x8_mode=t8, num_ref_idx_l0=l0,
                  num_ref_idx_l1=l1, gop_length=gop, slices_per_picture=spp, seed=90 + st + 3 * cf + t8)
    ps, verdict = _check_batch_against_oracle(ctx, data, require_all=True)
    assert len(ps.descs) == 3 * spp


@pytest.mark.parametrize("case", MBAFF_CASES[2:], ids=lambda c: "x".join(map(str, c)))
def test_mbaff_files_match_oracle(ctx, case, monkeypatch):
    monkeypatch.setenv("AVR_RMODE_PARALLEL", "1")   # the parallel R-mode compress, whatever the cost rule picks
    st, cf, t8, l0, l1, gop, spp = case
    data = _mbaff(ctx, 4, slice_type=st, chroma_format_idc=cf, transform_8x8_mode=t8, num_ref_idx_l0=l0,
                  num_ref_idx_l1=l1, gop_length=gop, slices_per_picture=spp, seed=120 + st + 3 * cf)
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "mbaff.264"
        f.write_bytes(data)
        for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL)):
            avrc = ctx.compress(data, model)
            assert avrc == oracle_cli("compress", f, mode=mode), mode
            assert ctx.decompress(avrc) == data
    os.environ["AVR_RMODE_SEQUENTIAL"] = "1"
    try:
        seq = ctx.compress(data, avr.MODEL_REFERENCE)
    finally:
        del os.environ["AVR_RMODE_SEQUENTIAL"]
    assert seq == ctx.compress(data, avr.MODEL_REFERENCE)


def test_progressive_field_and_mbaff_in_one_file(ctx):
    """Progressive, PAFF and MBAFF pictures of one size in one file (three SPS): the walker's
    field tables, model rows and pair storage switch per slice in one reference-model walk."""
    a = ctx.synthesize(avr.SynthParams(mb_width=10, mb_height=6, slice_type=0, slice_qp=26, seed=11, gop_length=2), 2)
    b = _paff(ctx, 2, mb_width=10, mb_height=6, slice_type=0, seed=12, gop_length=2)
    c = _mbaff(ctx, 2, mb_width=10, mb_height=6, slice_type=0, seed=13, gop_length=2)
    data = a + b + c + a
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "all.264"
        f.write_bytes(data)
        for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL)):
            avrc = ctx.compress(data, model)
            assert avrc == oracle_cli("compress", f, mode=mode), mode
            assert ctx.decompress(avrc) == data


@pytest.mark.parametrize("structure", [1, 2])
def test_damaged_field_slices_are_contained(ctx, structure):
    """Truncated and corrupted field / MBAFF slices end with status < 0 (stored skip_coded), never a
    fault; the undamaged ones round-trip; whole damaged files still compress and come back exactly
    in both model modes."""
    import numpy as np
    from avrecode_amd.batch import DeviceBatch
    data = ctx.synthesize(avr.SynthParams(mb_width=12, mb_height=8, slice_type=0, slice_qp=24, seed=31,
                                          structure=structure, gop_length=3, slices_per_picture=2), 3)
    ps = avr.parse_stream(data)
    rng = np.random.default_rng(9)
    d = ps.descs.copy()
    arena = ps.arena.copy()
    for k in range(len(d)):
        o, s = int(d[k]["payload_offset"]), int(d[k]["payload_size"])
        if k % 3 == 0:
            d[k]["payload_size"] = d[k]["read_limit"] = max(1, s // 2)
        elif k % 3 == 1:
            idx = rng.integers(o, o + s, size=8)
            arena[idx] ^= rng.integers(1, 256, size=8).astype(np.uint8)
    bad = avr.ParsedStream(d, arena, ps.work_len, ps.max_mb_width, ps.max_mb_height)
    b = DeviceBatch(ctx, bad)
    b.roundtrip(avr.MODEL_PARALLEL)
    torch.cuda.synchronize()
    v = b.verdicts()
    assert set(np.unique(v)) <= {1, 2}
    assert (v[0::3] == 2).all() and (v[2::3] == 1).all()
    # whole files with damaged bytes inside slice payloads
    raw = bytearray(data)
    for k in rng.integers(len(raw) // 4, len(raw), size=24):
        raw[int(k)] ^= 0x5A
    raw = bytes(raw)
    for model in (avr.MODEL_REFERENCE, avr.MODEL_PARALLEL):
        avrc = ctx.compress(raw, model)
        assert ctx.decompress(avrc) == raw


def test_field_lane_matches_serial_launch(ctx, monkeypatch):
    """A parallel batch of progressive and field slices runs the field kernel on a stream of its own
    beside the progressive one (the context's field lane, avr::FieldLane); AVR_FIELD_LANE=0 runs the
    two one after the other.  Both give the same containers, which decompress back: with the resident
    kernels (three files) and with the persistent queue kernels (more slices than resident slots, where
    the field kernel's workgroups take the estimator scratches after the progressive ones)."""
    prog = ctx.synthesize(avr.SynthParams(mb_width=8, mb_height=4, slice_type=0, slice_qp=26, seed=21, gop_length=3,
                                          slices_per_picture=4), 8)
    fld = _paff(ctx, 4, mb_width=8, mb_height=4, slice_type=0, seed=22, gop_length=3, slices_per_picture=4)
    mbf = _mbaff(ctx, 4, mb_width=8, mb_height=4, slice_type=1, seed=23, gop_length=3, slices_per_picture=2)
    small = [prog, fld, mbf]
    per_set = sum(len(avr.parse_stream(d).descs) for d in small)
    sets = 1
    while ctx.slice_kernel(sets * per_set, 8, False).startswith("slices_parallel_kernel"):
        sets *= 2
    assert sets > 1
    for files in (small, small * sets):
        on = ctx.compress_files(files, avr.MODEL_PARALLEL)
        assert ctx.decompress_files(on) == files
        monkeypatch.setenv("AVR_FIELD_LANE", "0")
        with avr.Context(0) as serial:
            assert serial.compress_files(files, avr.MODEL_PARALLEL) == on
        monkeypatch.delenv("AVR_FIELD_LANE")
