"""The product's recode.proto wire codec (avr_front.cpp pb_* through avr_container_describe and
avr_assemble_container) against the Python protobuf runtime (tests/_pb.py, recode.proto:1-19).

* every tests/golden/container.json case: the library parses the protobuf runtime's bytes to the
  same fields and re-serialises them byte-identical;
* whole-file containers the library assembles for both fixtures (per-slice outputs of the oracle
  standing in for the device's): the protobuf runtime parses them, re-serialises byte-identical,
  sees the reference's block grammar, and agrees with the library's own parse field by field.
"""
import json

import numpy as np
import pytest

import _pb
from _oracle import ROOT, slices_p

avr = pytest.importorskip("avrecode_amd")
CASES = json.loads((ROOT / "tests/golden/container.json").read_text())
FIX = ROOT / "tests" / "fixtures"


@pytest.mark.parametrize("i", range(len(CASES)))
def test_library_parses_runtime_bytes(i):
    case = CASES[i]
    raw = bytes.fromhex(case["bytes"])
    desc, again = avr.describe_container(raw)
    assert again == raw
    assert desc == _pb.describe(_pb.parse(raw))
    want_v = None if case["version"] is None else case["version"].encode().hex()
    assert desc["version"] == want_v
    assert len(desc["blocks"]) == len(case["blocks"])
    for got, want in zip(desc["blocks"], case["blocks"]):
        assert got == want


@pytest.mark.parametrize("blob", [b"\x12", b"\x12\x05\x08", b"\x0a\x80", b"\x12\x02\x22\x09"])
def test_library_rejects_truncated(blob):
    with pytest.raises(avr.AvrError):
        avr.describe_container(blob)


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_assembled_container_against_runtime(name):
    data = (FIX / name).read_bytes()
    _, recs = slices_p(data)
    st = np.array([0 if r["recodable"] else -1 for r in recs], np.int32)
    blobs = [r["recoded"] if r["recodable"] else b"" for r in recs]
    lens = np.array([len(b) for b in blobs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    avrc = avr.assemble_container(data, st, b"".join(blobs), offs, lens)
    m = _pb.check_container(avrc, data)
    assert m.metadata.version  # the parallel-model tag
    # coded blocks = the recodable slices whose payload occurs verbatim (EPB slices do not: they
    # are stored skip_coded, recode.cpp:1285-1296), in file order
    coded = [b.cabac for b in m.block if b.HasField("cabac")]
    cand = iter(x for x, s in zip(blobs, st) if s == 0)
    assert all(any(c == x for x in cand) for c in coded)
    assert len(coded) + sum(1 for b in m.block if b.HasField("skip_coded")) == len(recs)
    desc, again = avr.describe_container(avrc)
    assert again == avrc and desc == _pb.describe(m)
