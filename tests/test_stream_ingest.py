"""The streaming hooks session's incremental parser (host only, CPU): the bytes a caller's demuxer
feeds (avr_hooks_feed: the fork's read_packet, recode.cpp:1127-1131) are parsed as they arrive --
each Annex-B NAL unit once the next start code is in, each MP4 sample once the moov box and the
sample are in -- instead of re-parsing everything fed so far at every init_decoder (O(n^2) over a
stream).  Checked here through avr_debug_stream_slices (a debug export of libavrecode.so):

* fed in fixed-size pieces (1, 4, 32 KiB) or at random cut points, the slices found (NAL offset and
  size, payload size, picture id) equal parse_file's on the whole file, for Annex-B streams, a
  moov-last MP4 (nothing parses before the moov box at the end), and a moov-first ("faststart")
  MP4 -- which the whole-prefix demux used to reject at the first sample past the bytes fed;
* fed NAL unit by NAL unit with the decoder asking for each slice as soon as its unit is in (the
  unit in progress taken provisionally), the same slices; a unit that a later feed extends fails
  the parse (the decoder would have decoded a truncated slice).
"""
import ctypes

import numpy as np
import pytest

from _oracle import ROOT

import avrecode_amd as avr

FIX = ROOT / "tests" / "fixtures"


def _slices(data: bytes, cuts=None, provisional=False):
    L = avr.lib()
    f = L.avr_debug_stream_slices
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_int]
    cap = 4096
    out = np.zeros(4 * cap, np.uint64)
    c = np.asarray(cuts if cuts is not None else [len(data)], np.uint64)
    r = f(data, len(data), c.ctypes.data, len(c), 1 if cuts is not None else 0, 1 if provisional else 0,
          out.ctypes.data, cap)
    if r < 0:
        return r
    return [tuple(int(v) for v in out[4 * i:4 * i + 4]) for i in range(r)]


def _boxes(b: bytes, off: int = 0, end: int | None = None):
    end = len(b) if end is None else end
    while off + 8 <= end:
        size, typ, hdr = int.from_bytes(b[off:off + 4], "big"), b[off + 4:off + 8], 8
        if size == 1:
            size, hdr = int.from_bytes(b[off + 8:off + 16], "big"), 16
        elif size == 0:
            size = end - off
        yield typ, off, hdr, size
        off += size


def faststart(mp4: bytes) -> bytes:
    """The same MP4 with its moov box moved in front of the media data (what `-movflags faststart`
    writes): chunk offsets (stco / co64) shifted by the moov box's size."""
    top = list(_boxes(mp4))
    moov = next(t for t in top if t[0] == b"moov")
    m = bytearray(mp4[moov[1]:moov[1] + moov[3]])
    shift = len(m)

    def patch(off, end):
        for typ, o, hdr, size in _boxes(m, off, end):
            if typ in (b"trak", b"mdia", b"minf", b"stbl"):
                patch(o + hdr, o + size)
            elif typ in (b"stco", b"co64"):
                cnt = int.from_bytes(m[o + hdr + 4:o + hdr + 8], "big")
                w = 4 if typ == b"stco" else 8
                for k in range(cnt):
                    p = o + hdr + 8 + w * k
                    m[p:p + w] = (int.from_bytes(m[p:p + w], "big") + shift).to_bytes(w, "big")
    patch(8, len(m))
    first_media = next(t[1] for t in top if t[0] == b"mdat")
    assert moov[1] > first_media, "already moov-first"
    rest = b"".join(mp4[o:o + s] for t, o, h, s in top if o >= first_media and t != b"moov")
    return mp4[:first_media] + bytes(m) + rest


def _inputs():
    out = {n: (FIX / n).read_bytes() for n in ("realshort.mp4", "cockatoo.mp4", "paff_ipp.264", "mbaff_ib.264")}
    out["realshort_faststart.mp4"] = faststart(out["realshort.mp4"])
    return out


INPUTS = _inputs()


def test_faststart_file_parses_like_the_original():
    a, b = INPUTS["realshort.mp4"], INPUTS["realshort_faststart.mp4"]
    assert len(a) == len(b) and a != b
    sa, sb = _slices(a), _slices(b)
    assert len(sa) == len(sb) == 36
    assert [s[1:] for s in sa] == [s[1:] for s in sb]   # same NAL sizes, payloads, pictures
    assert avr.parse_stream(a).arena.tobytes() == avr.parse_stream(b).arena.tobytes()


@pytest.mark.parametrize("name", sorted(INPUTS))
@pytest.mark.parametrize("chunk", [1024, 4096, 32768, 0], ids=["1k", "4k", "32k", "random"])
def test_chunked_feed_parses_like_the_whole_file(name, chunk):
    data = INPUTS[name]
    if chunk:
        cuts = list(range(chunk, len(data), chunk)) + [len(data)]
    else:
        rng = np.random.default_rng(len(data))
        cuts = sorted(set(int(x) for x in rng.integers(1, len(data), size=60))) + [len(data)]
    assert _slices(data, cuts) == _slices(data)


@pytest.mark.parametrize("name", ["paff_ipp.264", "mbaff_ib.264"])
def test_nal_by_nal_feed_with_provisional_units(name):
    """Annex-B fed through the end of each NAL unit (start code of the next one not yet in), the
    decoder asking for the next slice each time: every slice is parsed as soon as its unit is in."""
    data = INPUTS[name]
    starts = []
    i = data.find(b"\x00\x00\x01")
    while i >= 0:
        starts.append(i)
        i = data.find(b"\x00\x00\x01", i + 3)
    ends = [s for s in starts[1:]] + [len(data)]
    # each cut: the unit's end without the next start code's leading zero bytes
    cuts = []
    for e in ends:
        while e > 0 and data[e - 1] == 0 and e != len(data):
            e -= 1
        cuts.append(e)
    assert _slices(data, cuts, provisional=True) == _slices(data)


def test_a_unit_extended_after_its_provisional_parse_fails():
    data = INPUTS["paff_ipp.264"]
    whole = _slices(data)
    nal_off, nal_size = whole[3][0], whole[3][1]
    cut = nal_off + nal_size // 2   # the decoder asks for slice 3 while half of its unit is in
    assert _slices(data, [cut, len(data)], provisional=True) == -3   # AVR_ERR_FORMAT
    assert _slices(data, [cut, len(data)], provisional=False) == whole  # not asked for early: fine
