"""Container assembly at stream scale (CPU, host only): BASELINE configs[3]'s rank-0 step.

find_next_coded_block_and_emit_literal (recode.cpp:1275-1297) searches each coded slice's unescaped
payload in the file after the previous coded block (memmem).  A payload whose NAL had
emulation-prevention bytes occurs nowhere, and memmem then scans to the end of the file -- once per
such slice, O(misses x file): the full-size 4.47 GB configs[3] stream did not get through one step
in 13 minutes.  avr_api.cpp's find_payload gives memmem's answer from an index of the file's
00 00 0y trigrams instead.  Checked here:

* the containers equal the ones the reference's search gives (Python bytes.find from the previous
  block's end, the same semantics), on streams built to hit every case: payloads with
  emulation-prevention bytes that occur nowhere, payloads whose unescaped bytes DO occur verbatim
  after the previous block (in a filler NAL right before their own slice), and payloads without a
  trigram (found in their own NAL);
* avr_assemble_container and avr_assemble_container_parsed (rank 0's own parse, no second pass)
  agree;
* assembly time grows linearly: a 4x longer stream takes <= 4.5x the time.
"""
import time

import numpy as np
import pytest

from _oracle import ROOT

import avrecode_amd as avr

FIX = ROOT / "tests" / "fixtures"


def _nals(stream: bytes):
    """(non-slice NAL units, slice NAL units) of an Annex-B stream, each with a 4-byte start code."""
    import bench
    return bench._split_slices(stream)


def _escape(raw: bytes) -> bytes:
    """H.264 emulation prevention (7.4.1): 00 00 0y (y <= 3) -> 00 00 03 0y."""
    out, zeros = bytearray(), 0
    for b in raw:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


def _stream(n_slices: int, seed: int, tail: bool = False) -> bytes:
    """A tiled Annex-B stream: the field fixture's parameter sets, then n_slices slices made from its
    first slice NAL with seeded bytes appended to the payload (kinds cycle: a run with 00 00 0y
    trigrams -> emulation-prevention bytes; the same, preceded by a filler NAL holding the slice's
    unescaped payload verbatim; plain bytes)."""
    head, slices = _nals((FIX / "paff_ipp.264").read_bytes())
    tmpl = slices[0]
    rng = np.random.default_rng(seed)
    out = [head]
    for i in range(n_slices):
        raw = bytearray(rng.integers(1, 256, size=int(rng.integers(3000, 9000)), dtype=np.uint8).tobytes())
        kind = i % 3
        if kind in (0, 1) and tail:
            # the payload's only trigram in its last six bytes (no four bytes after it to key on)
            at = len(raw) - int(rng.integers(2, 5))
            raw[at:at + 3] = bytes([0, 0, int(rng.integers(2, 4))])
            del raw[at + 3:]
        elif kind in (0, 1):
            for _ in range(3):
                at = int(rng.integers(16, len(raw) - 8))
                raw[at:at + 3] = bytes([0, 0, int(rng.integers(2, 4)) if kind == 1 else int(rng.integers(0, 4))])
        out.append(tmpl + _escape(bytes(raw) + b"\x80"))
    data = b"".join(out)
    # kind 1: a filler NAL (type 12) right before the slice holding its unescaped payload verbatim
    # (only 00 00 02 / 00 00 03 trigrams: no start code inside it)
    ps = avr.parse_stream(data)
    parts = [head]
    _, sl = _nals(data)
    for i, nal in enumerate(sl):
        if i % 3 == 1:
            d = ps.descs[i]
            pay = ps.arena[int(d["payload_offset"]):int(d["payload_offset"]) + int(d["payload_size"])].tobytes()
            parts.append(b"\x00\x00\x00\x01\x0c" + pay + b"\x80")
        parts.append(nal)
    return b"".join(parts)


def _expected_layout(data: bytes, ps, ok):
    """The reference's segmentation (memmem from the previous block's end, recode.cpp:1285)."""
    found, prev = [], 0
    for k, d in enumerate(ps.descs):
        size = int(d["payload_size"])
        if not ok[k] or size < 8:
            found.append(None)
            continue
        pay = ps.arena[int(d["payload_offset"]):int(d["payload_offset"]) + size].tobytes()
        f = data.find(pay, prev)
        found.append(f if f >= 0 else None)
        if f >= 0:
            prev = f + size
    return found


def _layout_of(avrc: bytes):
    desc, _ = avr.describe_container(avrc)
    pos, out = 0, []
    for b in desc["blocks"]:
        if "literal" in b:
            pos += len(b["literal"]) // 2
        elif "cabac" in b:
            out.append(pos)
            pos += b["size"]
        else:
            out.append(None)
    return out


def _assemble(data, ps, parsed: bool):
    n = len(ps.descs)
    st = np.where(ps.descs["coded"] == 1, 0, -1).astype(np.int32)
    lens = np.full(n, 5, np.uint32)
    offs = (np.arange(n, dtype=np.uint64) * 5).astype(np.uint64)
    blob = np.frombuffer(b"RCODE" * n, np.uint8)
    return avr.assemble_container(data, st, blob, offs, lens, ps=ps if parsed else None), st == 0


def test_segmentation_equals_reference_search():
    data = _stream(60, seed=1)
    ps = avr.parse_stream(data)
    assert len(ps.descs) == 60
    a, ok = _assemble(data, ps, parsed=True)
    b, _ = _assemble(data, ps, parsed=False)
    assert a == b
    exp = _expected_layout(data, ps, ok)
    assert _layout_of(a) == exp
    # every case occurs: not found (emulation prevention), found in a filler NAL, found in place
    kinds = {("miss" if f is None else "filler" if k % 3 == 1 else "own") for k, f in enumerate(exp) if ok[k]}
    assert kinds == {"miss", "filler", "own"}, kinds
    # the container restores the stream's layout (literals + coded sizes)
    desc, _ = avr.describe_container(a)
    assert sum(len(x.get("literal", "")) // 2 + (x["size"] if "cabac" in x else 0) for x in desc["blocks"]) == len(data)


def test_segmentation_unkeyed_trigrams():
    """Payloads whose only 00 00 0y trigram lies in their last six bytes (the index has no four
    following bytes to key on: find_payload's by-position lists): memmem's answer, found in the
    filler NAL or nowhere."""
    data = _stream(60, seed=3, tail=True)
    ps = avr.parse_stream(data)
    a, ok = _assemble(data, ps, parsed=True)
    exp = _expected_layout(data, ps, ok)
    assert _layout_of(a) == exp
    kinds = {("miss" if f is None else "filler" if k % 3 == 1 else "own") for k, f in enumerate(exp) if ok[k]}
    assert kinds == {"miss", "filler", "own"}, kinds


def test_parsed_assembly_checks_recorded_positions():
    """avr_assemble_container_parsed takes rank 0's parse: each payload's recorded file position is
    used only where the payload's bytes stand there.  An arena whose payload differs from the file
    in its middle bytes (a stale parse, another revision of the file) gets memmem's answer for the
    bytes it holds -- here: found nowhere, so the slice is a literal -- not a block at the recorded
    position that would decompress to other bytes."""
    import copy
    data = _stream(60, seed=4)
    ps = avr.parse_stream(data)
    ps2 = copy.copy(ps)
    ps2.arena = ps.arena.copy()
    changed = []
    for k in (2, 5, 11):   # kind 2: payloads found in their own NAL
        d = ps.descs[k]
        mid = int(d["payload_offset"]) + int(d["payload_size"]) // 2
        ps2.arena[mid] ^= 0x5A
        changed.append(k)
    a, ok = _assemble(data, ps2, parsed=True)
    exp = _expected_layout(data, ps2, ok)
    lay = _layout_of(a)
    assert lay == exp
    assert all(lay[k] is None for k in changed) and all(_expected_layout(data, ps, ok)[k] is not None for k in changed)


def test_assembly_scales_linearly():
    """A 4x longer stream (the same slices, with their filler NAL units, tiled four times) takes
    about 4x the time: no per-slice search that grows with the file.  Best of three runs each, with
    slack for timer and scheduler noise on a shared host."""
    def best_time(data, ps):
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            _assemble(data, ps, parsed=True)
            t.append(time.perf_counter() - t0)
        return min(t)
    small = _stream(900, seed=2)
    # the parameter sets once, then everything after them (slices and filler NAL units in their
    # order) four times: a long stream of one repeated GOP, as configs[3] is made
    ps_s = avr.parse_stream(small)
    body_at = small.index(b"\x00\x00\x00\x01", small.index(b"\x00\x00\x00\x01\x68") + 4)
    big = small[:body_at] + small[body_at:] * 4
    ps_b = avr.parse_stream(big)
    assert len(ps_b.descs) == 4 * len(ps_s.descs)
    ts, tb = best_time(small, ps_s), best_time(big, ps_b)
    assert tb <= 6 * ts + 0.05, (ts, tb)
