"""The parallel model's long-slice split, on the CPU oracle (oracle/oracle_seams.c; this library's
own format -- the reference decodes a slice as one chain, recode.cpp:1411-1520).  Parity of the
format itself: every piece of every split slice of the x264 fixtures, decompressed on its own from
its seam (the byte-form re-encoder state derived from the CABAC decoder's offset, the context states,
the upper row's edges), spliced at the seams' q, restores the payload; the whole-file oracle
roundtrip with the split restores the file; no field picture or MBAFF slice is ever cut."""
import json
import subprocess

import pytest

from _oracle import ROOT, build_oracle, oracle_cli

FIX = ROOT / "tests" / "fixtures"


def _pieces(path, split_bytes):
    _, cli = build_oracle()
    import os
    env = dict(os.environ, AVR_SPLIT_BYTES=str(split_bytes))
    r = subprocess.run([str(cli), "pieces", str(path)], capture_output=True, env=env)
    out = r.stdout.decode()
    f = out.split()
    return r.returncode, int(f[2]), int(f[4]), int(f[6])


@pytest.mark.parametrize("split_bytes", [384, 1024, 3000])
@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_every_piece_decompresses_alone(name, split_bytes):
    rc, split, pieces, bad = _pieces(FIX / name, split_bytes)
    assert rc == 0 and bad == 0
    assert split > 0 and pieces > split


@pytest.mark.parametrize("name", ["mbaff_ib.264", "paff_ipp.264"])
def test_field_slices_are_never_cut(name):
    rc, split, pieces, bad = _pieces(FIX / name, 256)
    assert rc == 0 and split == 0 and pieces == 0


@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
def test_oracle_roundtrip_with_split(tmp_path, name):
    data = (FIX / name).read_bytes()
    plain = oracle_cli("compress", FIX / name, mode="P", split_bytes=0)
    split = oracle_cli("compress", FIX / name, mode="P", split_bytes=1024)
    assert len(split) > len(plain)   # seams fields and fresh models cost bytes
    f = tmp_path / "s.avrc"
    f.write_bytes(split)
    assert oracle_cli("decompress", f) == data
    # the default split (96 KiB) leaves these small slices whole: the container is the plain one
    assert oracle_cli("compress", FIX / name, mode="P", split_bytes=98304) == plain


def test_split_container_has_seams_fields(tmp_path):
    """Block field 16 appears exactly on the cut blocks, through the product's own wire codec when
    it is importable (a host-only call: no GPU needed)."""
    split = oracle_cli("compress", FIX / "realshort.mp4", mode="P", split_bytes=1024)
    try:
        import avrecode_amd as avr
        info, again = avr.describe_container(split)
    except ImportError:
        pytest.skip("libavrecode.so not built")
    assert again == split   # field 16 parses and re-serialises byte for byte
    cut = [b for b in info["blocks"] if "seams" in b]
    assert cut and all("cabac" in b for b in cut)


def test_plans_refuse_split_containers():
    """The per-slice decompress paths (plans for sharded runs) cannot hand out pieces: they refuse a
    split container with AVR_ERR_UNSUPPORTED (-6); host-only calls, no GPU needed."""
    try:
        import avrecode_amd as avr
        avr.lib()
    except (ImportError, OSError):
        pytest.skip("libavrecode.so not built")
    split = oracle_cli("compress", FIX / "realshort.mp4", mode="P", split_bytes=1024)
    with pytest.raises(avr.AvrError) as e:
        avr.plan_decompress(split)
    assert e.value.code == -6
    with pytest.raises(avr.AvrError) as e:
        avr.DecompressPlan().load(split)
    assert e.value.code == -6
    plain = oracle_cli("compress", FIX / "realshort.mp4", mode="P", split_bytes=0)
    assert len(avr.plan_decompress(plain).descs) > 0
