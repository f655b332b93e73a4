"""recode.proto wire codec of the oracle against the Python protobuf runtime's serialisation."""
import ctypes
import json

import pytest

from _oracle import ROOT

CASES = json.loads((ROOT / "tests/golden/container.json").read_text())


def _pb_varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def python_restatement(case):
    """Independent proto2 writer (field-number order, presence kept) used to cross-check."""
    out = bytearray()
    if case["version"] is not None:
        v = case["version"].encode()
        md = b"\x0a" + _pb_varint(len(v)) + v
        out += b"\x0a" + _pb_varint(len(md)) + md
    for b in case["blocks"]:
        m = bytearray()
        if "size" in b:
            m += b"\x08" + _pb_varint(b["size"])
        if "literal" in b:
            lit = bytes.fromhex(b["literal"])
            m += b"\x12" + _pb_varint(len(lit)) + lit
        if "skip_coded" in b:
            m += b"\x18" + _pb_varint(int(b["skip_coded"]))
        if "cabac" in b:
            c = bytes.fromhex(b["cabac"])
            m += b"\x22" + _pb_varint(len(c)) + c
        if "length_parity" in b:
            m += b"\x28" + _pb_varint(int(b["length_parity"]))
        if "last_byte" in b:
            lb = bytes.fromhex(b["last_byte"])
            m += b"\x32" + _pb_varint(len(lb)) + lb
        out += b"\x12" + _pb_varint(len(m)) + m
    return bytes(out)


@pytest.mark.parametrize("i", range(len(CASES)))
def test_golden_serialisation(i):
    assert python_restatement(CASES[i]).hex() == CASES[i]["bytes"]


def test_survey_probe_bytes():
    # empty literal -> 12 00; cabac block -> 08 e8 07 22 02 12 34 28 00 32 01 80
    assert CASES[0]["bytes"] == "12021200"
    assert CASES[1]["bytes"] == "120c08e80722021234280032" + "0180"
    assert CASES[2]["bytes"] == "1204080518" + "01"
