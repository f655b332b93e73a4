"""avr_parse_stream's max_mb_width covers the slices the device walks, not the ones it stores
skip_coded (CPU).

recodable_candidate marks an MBAFF slice whose neighbour ring (3 W + 7 records) overflows a
workgroup's LDS as uncoded, so the container stores it skip_coded (recode.cpp:1285-1296).  The
width that parse_stream reports sizes the DeviceBatch / sharded_compress launch: counting an
uncoded slice there would make the whole launch ask for more LDS than a CU has.  The stream here
is mbaff_ib.264 with its SPS's pic_width_in_mbs_minus1 rewritten to a 4K-plus width (the slice
headers still parse; the slice data is never walked).
"""
from _oracle import ROOT

import avrecode_amd as avr

FIX = ROOT / "tests" / "fixtures"


class _Bits:
    def __init__(self, rbsp: bytes):
        self.b, self.pos = rbsp, 0

    def u(self, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.b[self.pos >> 3] >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v

    def ue(self):
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)

    def se(self):
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


def _unescape(ebsp: bytes) -> bytes:
    return ebsp.replace(b"\x00\x00\x03", b"\x00\x00")


def _escape(rbsp: bytes) -> bytes:
    out, zeros = bytearray(), 0
    for c in rbsp:
        if zeros >= 2 and c <= 3:
            out.append(3)
            zeros = 0
        out.append(c)
        zeros = zeros + 1 if c == 0 else 0
    return bytes(out)


def _ue_bits(v: int) -> str:
    s = bin(v + 1)[2:]
    return "0" * (len(s) - 1) + s


def widen_sps(sps_rbsp: bytes, mb_width: int) -> bytes:
    """The SPS with pic_width_in_mbs_minus1 = mb_width - 1 (H.264 7.3.2.1.1), other fields kept."""
    r = _Bits(sps_rbsp)
    profile = r.u(8)
    r.u(16)
    r.ue()
    if profile in (100, 110, 122, 244, 44, 83, 86, 118, 128, 138, 139, 134, 135):
        if r.ue() == 3:
            r.u(1)
        r.ue(), r.ue(), r.u(1)
        if r.u(1):
            raise NotImplementedError("scaling lists")
    r.ue()
    poc = r.ue()
    if poc == 0:
        r.ue()
    elif poc == 1:
        r.u(1), r.se(), r.se()
        for _ in range(r.ue()):
            r.se()
    r.ue(), r.u(1)
    start = r.pos
    r.ue()
    bits = "".join(f"{c:08b}" for c in sps_rbsp)
    # the trailing bits (rbsp_stop_one_bit + alignment) move with the rest; re-pad to a byte
    body = bits[:start] + _ue_bits(mb_width - 1) + bits[r.pos:].rstrip("0")
    body += "0" * (-len(body) % 8)
    return bytes(int(body[i:i + 8], 2) for i in range(0, len(body), 8))


def _wide(data: bytes, mb_width: int) -> bytes:
    out, i = bytearray(), 0
    starts = []
    j = data.find(b"\x00\x00\x01")
    while j >= 0:
        starts.append(j + 3)
        j = data.find(b"\x00\x00\x01", j + 3)
    for k, s in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else len(data)
        nal = data[s:e]
        if nal[0] & 0x1F == 7:
            out += data[i:s] + nal[:1] + _escape(widen_sps(_unescape(nal[1:]), mb_width))
            i = e
    return bytes(out + data[i:])


def test_wide_mbaff_slices_are_uncoded_and_do_not_size_the_ring():
    data = (FIX / "mbaff_ib.264").read_bytes()
    base = avr.parse_stream(data)
    assert len(base.descs) > 0 and all(int(c) for c in base.descs["coded"])
    wide = avr.parse_stream(_wide(data, 600))   # ring 3 * 600 + 7 records: over 160 KiB
    assert len(wide.descs) == len(base.descs)
    assert (wide.descs["mb_width"] == 600).all()
    assert not any(int(c) for c in wide.descs["coded"])
    assert wide.max_mb_width <= base.max_mb_width


def test_widened_sps_keeps_the_other_fields():
    data = (FIX / "mbaff_ib.264").read_bytes()
    base, same = avr.parse_stream(data), avr.parse_stream(_wide(data, int(avr.parse_stream(data).descs["mb_width"][0])))
    assert same.arena.tobytes() == base.arena.tobytes()
    # every field but the payloads' file positions (the rewritten SPS may change its length)
    fields = [f for f in base.descs.dtype.names if f != "file_offset"]
    for f in fields:
        assert (same.descs[f] == base.descs[f]).all(), f
