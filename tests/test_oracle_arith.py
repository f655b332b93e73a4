"""The oracle's arithmetic coders against golden vectors produced by the reference's own
arithmetic_code.h compiled as-is (tests/golden/make_golden.py, oracle/ref_arith_driver.cpp)."""
import json
import random
import shutil
import subprocess
from pathlib import Path

import pytest

from _oracle import ROOT, lps_table, script_decode_ok, script_encode

GOLD = ROOT / "tests" / "golden"


def _load(name):
    return json.loads((GOLD / name).read_text())


@pytest.mark.parametrize("case", _load("arith_recoded.json"), ids=lambda c: f"seed{c['seed']}")
def test_recoded_coder_matches_reference(case):
    ops = [tuple(o) for o in case["ops"]]
    out = script_encode("recoded", ops)
    assert out.hex() == case["expect"]
    nsym = sum(1 for o in ops if o[0] == "s")
    assert script_decode_ok("recoded", out, ops) == nsym


@pytest.mark.parametrize("case", _load("arith_cabac.json"), ids=lambda c: f"seed{c['seed']}")
def test_cabac_encoder_matches_reference(case):
    ops = [tuple(o) for o in case["ops"]]
    out = script_encode("cabac", ops)
    assert out.hex() == case["expect"]


@pytest.mark.parametrize("case", _load("arith_cabac.json"), ids=lambda c: f"seed{c['seed']}")
def test_cabac_encoder_decodes_with_spec_engine(case):
    """test/arithmetic_code.cpp:14-47 / 66-91: the CABAC re-encoder's output must be read back
    bin-for-bin by the H.264 decoding engine (the #if 0 cross-checks of the reference test)."""
    ops = [tuple(o) for o in case["ops"]]
    out = script_encode("cabac", ops)
    n = sum(1 for o in ops if o[0] in "dbt")
    assert script_decode_ok("cabac", out, ops) == n


def test_recoded_roundtrip_half_probability():
    """test/arithmetic_code.cpp:93-111: random bits at p = 1/2 round-trip."""
    rng = random.Random(0)
    ops = [("s", rng.randint(0, 1), 1, 1) for _ in range(5000)] + [("f", 0, 0, 0)]
    out = script_encode("recoded", ops)
    assert script_decode_ok("recoded", out, ops) == 5000
    assert 600 <= len(out) <= 640  # ~1 bit per symbol


def test_lps_table_spot_values():
    t = lps_table()
    # rangeTabLPS[0][*] = 128 176 208 240; [63][*] = 2; duplicated for both valMPS
    assert [t[q * 128] for q in range(4)] == [128, 176, 208, 240]
    assert t[1] == t[0] and all(t[q * 128 + 126] == 2 for q in range(4))


@pytest.mark.skipif(not Path("/root/reference/arithmetic_code.h").exists(), reason="reference not mounted")
def test_live_reference_random_scripts():
    """Fresh seeds straight against the reference header compiled here (build container only)."""
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "ref"], check=True)
    ref = ROOT / "oracle" / "_ref" / "ref_arith"
    rng = random.Random(1234)
    for trial in range(4):
        ops = []
        for _ in range(4000):
            pos, neg = rng.randint(1, 0x60), rng.randint(1, 0x60)
            ops.append(("s", int(rng.random() < pos / (pos + neg)), pos, neg))
        ops.append(("f", 0, 0, 0))
        text = "recoded\n" + "\n".join(f"s {a} {b} {c}" if o == "s" else "f" for o, a, b, c in ops) + "\n"
        r = subprocess.run([str(ref)], input=text, capture_output=True, text=True, check=True)
        assert r.stdout.split()[0] == script_encode("recoded", ops).hex()
