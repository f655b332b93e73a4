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


# --------------------------------------------------------------------------- P-format coder
# The parallel model's container ("avrecode-amd:P32") is this library's own format: its coder
# has no reference implementation to be pinned against.  It is pinned here against an
# independent restatement in exact integer arithmetic (the whole coded value as one Python int),
# and the GPU's P-mode output is pinned against the oracle by the -m gpu parity tests.
def _p1(rng_, pos, neg):
    return ((rng_ * ((1 << 32) // (pos + neg))) >> 32) * pos


def _p_encode_bigint(ops):
    low, rng_, k = 0, 0xFFFFFFFF, 0
    for op in ops:
        if op[0] != "s":
            continue
        r1 = _p1(rng_, op[2], op[3])
        r0 = rng_ - r1
        assert r1 > 0 and r0 > 0
        if op[1]:
            low += r0
            rng_ = r1
        else:
            rng_ = r0
        if rng_ < 1 << 24:
            low, rng_, k = low << 8, rng_ << 8, k + 1
    sb = 1 << 31
    while sb:
        x = (low | sb) & ~(sb - 1)
        if sb < rng_ and low <= x < low + rng_:
            low = x
            break
        sb >>= 1
    return low.to_bytes(k + 4, "big").rstrip(b"\0")


def _p_scripts():
    out = []
    for seed, n, skew in [(21, 0, 0), (22, 1, 0), (23, 300, 0), (24, 5000, 0), (25, 5000, 1), (26, 40000, 2)]:
        rng = random.Random(seed)
        ops = []
        for _ in range(n):
            if skew == 2:
                pos, neg = rng.choice([(1, 95), (95, 1), (48, 48), (1, 1)])
            else:
                pos, neg = rng.randint(1, 0x60), rng.randint(1, 0x60)
            p = pos / (pos + neg)
            ops.append(("s", int(rng.random() < (p if skew != 1 else 1 - p)), pos, neg))
        out.append((seed, ops + [("f", 0, 0, 0)]))
    return out


@pytest.mark.parametrize("seed,ops", _p_scripts(), ids=lambda v: str(v) if isinstance(v, int) else "")
def test_p_coder_matches_exact_restatement(seed, ops):
    out = script_encode("p", ops)
    assert out == _p_encode_bigint(ops)
    assert script_decode_ok("p", out, ops) == sum(1 for o in ops if o[0] == "s")


def test_p_coder_costs_no_more_than_the_reference_coder():
    """The 32-bit coder's truncated quotient costs < 1e-5 bit per decision: within a few bytes
    of the reference's arithmetic_code<uint64_t, uint8_t> on the same decisions."""
    for seed, ops in _p_scripts()[3:]:
        p, r = script_encode("p", ops), script_encode("recoded", ops)
        assert len(p) <= len(r) + 4, (seed, len(p), len(r))


def test_p_coder_carry_chain():
    # a run of near-certain ones after a long run of 0xFF digits forces carries through them
    ops = [("s", 0, 1, 96)] * 3000 + [("s", 1, 1, 96)] * 20 + [("s", 1, 96, 1)] * 5000 + [("f", 0, 0, 0)]
    out = script_encode("p", ops)
    assert out == _p_encode_bigint(ops)
    assert script_decode_ok("p", out, ops) == len(ops) - 1
