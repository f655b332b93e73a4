"""Real-stream known answers (x264 CABAC fixtures, tests/fixtures/):
every slice parses to end_of_slice, regenerates its CABAC payload exactly, and whole files
round-trip bit-exactly in both model modes; the .avrc bytes are pinned in fixtures.json."""
import hashlib
import json
import subprocess

import pytest

from _oracle import ROOT, build_oracle, oracle_cli

FIX = ROOT / "tests" / "fixtures"


@pytest.mark.parametrize("name,nslices", [("realshort.mp4", 36), ("cockatoo.mp4", 280)])
def test_every_slice_regenerates(name, nslices):
    _, cli = build_oracle()
    r = subprocess.run([str(cli), "slices", str(FIX / name)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert f"slices ok {nslices} bad 0" in r.stdout


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
@pytest.mark.parametrize("mode", ["R", "P", "C"])
def test_roundtrip_and_golden(name, mode):
    out = oracle_cli("roundtrip", FIX / name, mode=mode)
    assert b"roundtrip succeeded" in out
    avrc = oracle_cli("compress", FIX / name, mode=mode)
    gold = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}
    g = gold[(name, mode)]
    assert len(avrc) == g["avrc_len"]
    assert hashlib.sha256(avrc).hexdigest() == g["avrc_sha256"]


def test_reference_8x8_ordering_cannot_roundtrip(monkeypatch):
    """Documented reference bug: with the reference's decompressor ordering (nnz bits decoded
    before end_coding_type sets is_8x8, recode.cpp:1476-1480 vs 1204-1212) 8x8-transform streams
    do not round-trip.  The oracle (and the product) key the decompressor like the compressor."""
    _, cli = build_oracle()
    env = dict(**__import__("os").environ, AVR_REFERENCE_8X8_BUG="1")
    r = subprocess.run([str(cli), "roundtrip", str(FIX / "realshort.mp4")], capture_output=True, env=env)
    assert r.returncode != 0


FIELDS = json.loads((ROOT / "tests/golden/fields.json").read_text())["files"]


@pytest.mark.parametrize("g", FIELDS, ids=lambda g: g["file"])
def test_field_fixture_regenerates_and_roundtrips(g):
    """Field pictures (PAFF) and MBAFF frames (tests/golden/fields.json): every slice parses to
    end_of_slice and regenerates its payload (field ctxIdx offsets, 8x8 field map, macroblock-pair
    neighbours of Table 6-4, oracle_walker.c), and whole-file compress in both model modes
    round-trips to the pinned containers."""
    _, cli = build_oracle()
    f = FIX / g["file"]
    r = subprocess.run([str(cli), "slices", str(f)], capture_output=True, text=True)
    assert r.returncode == 0 and f"slices ok {g['slices']} bad 0" in r.stdout, r.stdout[-2000:]
    for mode in ("R", "P", "C"):
        assert b"roundtrip succeeded" in oracle_cli("roundtrip", f, mode=mode)
        avrc = oracle_cli("compress", f, mode=mode)
        assert len(avrc) == g[mode]["avrc_len"]
        assert hashlib.sha256(avrc).hexdigest() == g[mode]["avrc_sha256"]


def _tiled_paff(copies=5):
    """The PAFF fixture's slices tiled (every copy restarts at its IDR picture): 8 * copies slices,
    so the chained model (AVR_CHAIN_SLICES = 16) cuts it into several chains."""
    import bench
    head, sl = bench._split_slices((FIX / "paff_ipp.264").read_bytes())
    return head, sl * copies


@pytest.mark.parametrize("lead", [0, 3], ids=["idr_aligned", "mid_gop"])
def test_chained_model_is_the_reference_model_per_chain(tmp_path, lead):
    """The chained model ("avrecode-amd:R16") is the reference model restarted every 16 coded slices:
    chain j's re-coded blocks equal the reference model's blocks for a file made of the parameter
    sets and chain j's slices alone (recode.cpp:1057's fresh estimators and update_frame_spec's fresh
    frames at that file's start), so the chained format is pinned wherever the reference model is."""
    import avrecode_amd as avr
    head, sl = _tiled_paff()
    # lead > 0: the first GOP's first `lead` slices again before the tiles (they are a valid start:
    # the IDR field pair and a P field), so the chain boundaries fall on P fields inside a GOP
    sl = sl[:lead] + sl
    data = head + b"".join(sl)
    f = tmp_path / "tiled.264"
    f.write_bytes(data)
    assert b"roundtrip succeeded" in oracle_cli("roundtrip", f, mode="C")
    blocks = [b["cabac"] for b in avr.describe_container(oracle_cli("compress", f, mode="C"))[0]["blocks"] if "cabac" in b]
    assert len(blocks) == len(sl) == 40 + lead
    whole_r = [b["cabac"] for b in avr.describe_container(oracle_cli("compress", f, mode="R"))[0]["blocks"] if "cabac" in b]
    assert blocks[:16] == whole_r[:16] and blocks[16:] != whole_r[16:]
    for j in range(0, len(sl), 16):
        g = tmp_path / f"chain{j}.264"
        g.write_bytes(head + b"".join(sl[j:j + 16]))
        sub = [b["cabac"] for b in avr.describe_container(oracle_cli("compress", g, mode="R"))[0]["blocks"] if "cabac" in b]
        assert blocks[j:j + 16] == sub, j


@pytest.mark.parametrize("name", ["realshort.mp4", "paff_ipp.264"])
def test_chained_family_ends_are_the_parallel_and_reference_models(tmp_path, name):
    """Chains of one coded slice are the parallel model (a fresh model per slice), one chain over the
    whole file is the reference model: the chained format sits between the two, and its re-coded
    blocks equal theirs at both ends (AVR_ORACLE_CHAIN overrides the chain length of 16, oracle only)."""
    import os
    import avrecode_amd as avr
    _, cli = build_oracle()

    def blocks(mode, k=None):
        o = tmp_path / f"{mode}{k}.avrc"
        env = dict(os.environ, **({"AVR_ORACLE_CHAIN": str(k)} if k else {}))
        flag = {"R": [], "P": ["-p"], "C": ["-c"]}[mode]
        subprocess.run([str(cli), "compress"] + flag + [str(FIX / name), str(o)], check=True, env=env)
        return [b["cabac"] for b in avr.describe_container(o.read_bytes())[0]["blocks"] if "cabac" in b]

    assert blocks("C", 1) == blocks("P")
    assert blocks("C", 1 << 30) == blocks("R")
