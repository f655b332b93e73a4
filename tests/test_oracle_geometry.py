"""Row a17 (get_neighbor_sub_mb + scan_8 / reverse_scan_8, recode.cpp:233-471) pinned by the
reference itself: tests/golden/geometry.json is the output of those lines of recode.cpp compiled
as-is (oracle/_ref/ref_geometry, tests/golden/make_geometry_golden.py).  Checked here against
  * the oracle's restatement (oracle_model.c, which derives reverse_scan_8 from scan_8), and
  * the neighbour table the library builds and the kernels load into LDS (HotTables::nb_left /
    nb_up, read by Walker::nz_bits), applied the way the walker applies it.
The device copy of the same table is compared in tests/test_gpu_parity.py."""
import ctypes
import json

import pytest

import avrecode_amd as avr
from _oracle import ROOT, lib as oracle_lib

GOLD = json.loads((ROOT / "tests" / "golden" / "geometry.json").read_text())


def test_reference_self_check_passed():
    # test_reverse_scan8() (recode.cpp:396-410) returned 0 in the reference build
    assert GOLD["test_reverse_scan8"] == 0
    assert len(GOLD["neighbors"]) == 2 * 5 * 51 * 4


def test_oracle_scan8_table_matches_reference():
    L = oracle_lib()
    L.oracle_scan_8.restype = ctypes.POINTER(ctypes.c_uint8)
    s = L.oracle_scan_8()
    assert [s[i] for i in range(51)] == GOLD["scan_8"]


def test_oracle_neighbors_match_reference():
    L = oracle_lib()
    fn = L.oracle_get_neighbor_sub_mb
    fn.restype = ctypes.c_int
    out = (ctypes.c_int * 3)()
    bad = []
    for above, size, idx, x, y, ok, ox, oy, oidx in GOLD["neighbors"]:
        r = fn(above, size, x, y, idx, out)
        got = (r, out[0], out[1], out[2])
        if got != (ok, ox, oy, oidx):
            bad.append(((above, size, idx, x, y), got, (ok, ox, oy, oidx)))
    assert not bad, bad[:5]


def walker_neighbor(nb_left: bytes, nb_up: bytes, above, size, idx, x, y):
    """The neighbour Walker::nz_bits derives from the LDS table (avr_walker.h, nz_bits): block n's
    left / upper block from nb_left / nb_up (| 128 = in the neighbouring macroblock), rounded down
    to a multiple of 4 for 8x8 blocks; DC blocks (n >= 48) take the same slot of the neighbour."""
    if idx >= 48:
        if above:
            return (1, x, y - 1, idx) if y > 0 else (0, x, y, idx)
        return (1, x - 1, y, idx) if x > 0 else (0, x, y, idx)
    e = (nb_up if above else nb_left)[idx]
    j = e & 63
    if size >= 32:
        j &= ~3
    cross = bool(e & 128)
    if cross and (y if above else x) == 0:
        return (0, x, y, idx)
    if cross:
        return (1, x, y - 1, j) if above else (1, x - 1, y, j)
    return (1, x, y, j)


def check_table(nb_left, nb_up):
    bad = []
    for above, size, idx, x, y, ok, ox, oy, oidx in GOLD["neighbors"]:
        got = walker_neighbor(nb_left, nb_up, above, size, idx, x, y)
        if got != (ok, ox, oy, oidx):
            bad.append(((above, size, idx, x, y), got, (ok, ox, oy, oidx)))
    return bad


def test_library_neighbor_table_matches_reference():
    nb_left, nb_up = avr.neighbor_tables(None)
    bad = check_table(nb_left, nb_up)
    assert not bad, bad[:5]


def test_table_check_detects_a_wrong_entry():
    nb_left, nb_up = avr.neighbor_tables(None)
    broken = bytearray(nb_up)
    broken[5] ^= 1
    assert check_table(nb_left, bytes(broken))


def test_upper_neighbours_read_only_the_kept_model_row_dwords():
    """The parallel model's walkers keep, per macroblock column, only the model bytes an upper
    neighbour lookup can reach (avr_walker.h kMringUsed: mnnz dwords 2, 3, 6, 7, 10, 11, 12).
    Pinned by the reference's own answer: every upper neighbour recode.cpp:233-471 returns in the
    macroblock above (tests/golden/geometry.json) lies in those dwords."""
    kept = {2, 3, 6, 7, 10, 11, 12}
    assert sum(1 << d for d in kept) == 0x1CCC
    reached = {oidx // 4 for above, size, idx, x, y, ok, ox, oy, oidx in GOLD["neighbors"]
               if above and ok and oy == y - 1}
    assert reached and reached <= kept, sorted(reached - kept)
