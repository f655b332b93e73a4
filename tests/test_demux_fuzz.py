"""Malformed inputs through the host front end (avr_front.cpp demux + parameter sets + slice
headers, via avr_parse_stream): truncated files, corrupted MP4 boxes (zero / backwards stsc chunk
numbers, 64-bit box sizes that would wrap, oversized counts) and corrupted SPS fields.  Every case
must return a status (AvrError) or a parse -- never crash, hang or read out of bounds.  Host only.
The reference's demuxer is libavformat (recode.cpp:73-135), absent here; these cases pin the
build's own front end, which every compress call runs before anything else."""
import random
import struct

import pytest

from _oracle import ROOT

avr = pytest.importorskip("avrecode_amd")
FIX = ROOT / "tests" / "fixtures"


def _parse(data):
    try:
        ps = avr.parse_stream(data)
    except avr.AvrError:
        return None
    for d in ps.descs:   # whatever parsed must describe payloads inside the arena
        assert int(d["payload_offset"]) + int(d["read_limit"]) <= len(ps.arena)
    return ps


def _box(data, name):
    i = data.find(name)
    assert i >= 4
    return i - 4


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_truncations(name):
    data = (FIX / name).read_bytes()
    rng = random.Random(1)
    cuts = sorted({rng.randrange(len(data)) for _ in range(24)} | {0, 1, 7, 8, 16, len(data) - 1})
    moov = _box(data, b"moov")
    cuts += [moov + k for k in (4, 8, 9, 100, 500)]
    for c in cuts:
        _parse(data[:c])


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_random_corruption_of_moov(name):
    data = (FIX / name).read_bytes()
    moov = _box(data, b"moov")
    rng = random.Random(2)
    for _ in range(60):
        b = bytearray(data)
        for _ in range(rng.randrange(1, 6)):
            b[rng.randrange(moov, len(b))] = rng.randrange(256)
        _parse(bytes(b))


def test_stsc_first_chunk_zero_and_backwards():
    data = (FIX / "realshort.mp4").read_bytes()
    s = _box(data, b"stsc")
    n = struct.unpack(">I", data[s + 12:s + 16])[0]
    assert n >= 1
    b = bytearray(data)
    b[s + 16:s + 20] = struct.pack(">I", 0)          # first_chunk of entry 0 = 0
    assert _parse(bytes(b)) is None
    b = bytearray(data)
    b[s + 16:s + 20] = struct.pack(">I", 0xFFFFFFFF)  # far past the last chunk
    _parse(bytes(b))


def test_box_with_wrapping_64bit_size():
    data = (FIX / "realshort.mp4").read_bytes()
    for name in (b"moov", b"trak", b"stbl", b"hdlr"):
        i = _box(data, name)
        b = bytearray(data)
        # size == 1: a 64-bit size follows the type; make off + size wrap past 2^64
        b[i:i + 4] = struct.pack(">I", 1)
        b[i + 8:i + 16] = struct.pack(">Q", 0xFFFFFFFFFFFFFFF8)
        _parse(bytes(b))
        b = bytearray(data)
        b[i:i + 4] = struct.pack(">I", 0xFFFFFFF0)     # 32-bit size past the end
        _parse(bytes(b))


def test_oversized_counts():
    data = (FIX / "realshort.mp4").read_bytes()
    for name, off in ((b"stsz", 20), (b"stco", 12), (b"stsc", 12)):
        i = _box(data, name)
        b = bytearray(data)
        b[i + off:i + off + 4] = struct.pack(">I", 0x7FFFFFFF)
        _parse(bytes(b))


def _annexb_with_sps(sps_rbsp: bytes) -> bytes:
    return b"\x00\x00\x00\x01\x67" + sps_rbsp + b"\x00\x00\x00\x01\x68\xee\x3c\x80"


def test_corrupt_sps_fields():
    # profile 66, level 30, then ue fields: an all-zero run makes every ue() take 31+ leading zeros
    for tail in (b"\x00" * 12, b"\x80" + b"\x00" * 8, b"\xff" * 16, b"\x00\x00\x00\x01" * 4):
        _parse(_annexb_with_sps(b"\x42\x00\x1e" + tail))
    # a synthetic stream's SPS with log2_max_frame_num and the picture size patched out of range
    ps = _parse(b"\x00\x00\x00\x01\x67\x42\x00\x1e\xf4\x02\x80\x2d\xc8")
    assert ps is None or len(ps.descs) == 0
