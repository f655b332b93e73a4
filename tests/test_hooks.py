"""The libavcodec-hooks callback surface of the C ABI (avr_hook_*, include/avrecode.h;
reference: AVCodecHooks trampolines recode.cpp:137-228).

tests/native/hooks_driver.c plays the fork's H.264 decoder with the oracle's slice_data() parser:
every bin of every re-coded slice is pulled through avr_hook_get / _bypass / _terminate and every
model event is reported, the parse being driven by the device's bins.  Compress through the hooks
must give the same container as the golden .avrc; decompress through the hooks must give the
original file back.
"""
import ctypes
import hashlib
import json
import subprocess
from functools import lru_cache

import pytest

from _oracle import ROOT, build_oracle

FIX = ROOT / "tests" / "fixtures"
GOLD = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}
BUILD = ROOT / "tests" / "native" / "_build"


@lru_cache(None)
def driver_path():
    build_oracle()
    lib = ROOT / "avrecode_amd" / "libavrecode.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(ROOT / "avrecode_amd"), "-j8"], check=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    out = BUILD / "libhooks_driver.so"
    src = ROOT / "tests" / "native" / "hooks_driver.c"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-Wall", str(src), "-o", str(out),
                    "-L" + str(ROOT / "oracle"), "-loracle", "-Wl,-rpath," + str(ROOT / "oracle"),
                    "-L" + str(ROOT / "avrecode_amd"), "-lavrecode", "-Wl,-rpath," + str(ROOT / "avrecode_amd")],
                   check=True)
    return out


def test_hooks_driver_builds_and_links():
    """CPU: the driver compiles against include/avrecode.h and links every avr_hook_* symbol."""
    L = ctypes.CDLL(str(driver_path()))
    assert L.hooks_compress and L.hooks_decompress and L.hooks_compress_stream and L.hooks_slice_regen


def _driver():
    L = ctypes.CDLL(str(driver_path()))
    pp = ctypes.POINTER(ctypes.c_uint8)
    L.hooks_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(pp),
                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_long)]
    L.hooks_compress_stream.argtypes = L.hooks_compress.argtypes
    L.hooks_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(pp),
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_long)]
    return L, pp


def _call(fn, *args):
    L, pp = _driver()
    out, n, walked = pp(), ctypes.c_size_t(), ctypes.c_long()
    r = getattr(L, fn)(*args, ctypes.byref(out), ctypes.byref(n), ctypes.byref(walked))
    data = ctypes.string_at(out, n.value) if r == 0 else b""
    if r == 0:
        import avrecode_amd as avr
        avr.lib().avr_free(out)
    return r, data, walked.value


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["realshort.mp4", "cockatoo.mp4"])
@pytest.mark.parametrize("mode,model", [("R", 0), ("P", 1)])
def test_hooks_compress_then_decompress(name, mode, model):
    data = (FIX / name).read_bytes()
    r, avrc, walked = _call("hooks_compress", data, len(data), model)
    assert r == 0, r
    g = GOLD[(name, mode)]
    assert hashlib.sha256(avrc).hexdigest() == g["avrc_sha256"]
    assert walked > 0
    r, back, walked_d = _call("hooks_decompress", avrc, len(avrc))
    assert r == 0, r
    assert walked_d == walked
    assert back == data


@pytest.mark.gpu
@pytest.mark.parametrize("model", [0, 1, 2, 3], ids=["R", "P64", "P32", "C"])
def test_hooks_decompress_on_demand(model):
    """A parallel-model container through the hooks is decoded on demand, as the reference's
    decompressor decodes each slice when FFmpeg reaches it (recode.cpp:1411-1520): nothing is
    regenerated before the first init_decoder, each init_decoder that reaches a slice not yet
    regenerated runs one device batch (that slice and at most 31 coded slices after it), and
    avr_hooks_end still returns the original file.  A reference-model container (whole or chained)
    is regenerated whole at begin (its estimators chain across slices): the debug count reads -1."""
    data = (FIX / "cockatoo.mp4").read_bytes()
    r, avrc, walked = _call("hooks_compress", data, len(data), model)
    assert r == 0, r
    r, back, walked_d = _call("hooks_decompress", avrc, len(avrc))
    assert r == 0, r
    assert back == data and walked_d == walked
    L, _ = _driver()
    buf = (ctypes.c_long * 4096)()
    n = L.hooks_slice_regen(buf, 4096)
    regen = list(buf[:n])
    assert n == 280   # cockatoo's slices, one init_decoder each
    if model in (0, 3):   # the reference model, whole or in chains: regenerated at begin
        assert set(regen) == {-1}
        return
    assert 0 < regen[0] <= 32
    assert regen == sorted(regen)
    assert regen[-1] == walked   # every re-coded slice, the last ones reached at the end
    steps = [b - a for a, b in zip(regen, regen[1:]) if b != a]
    assert steps and max(steps) <= 32 and len(steps) >= walked // 32 - 1


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["paff_ipp.264", "mbaff_ib.264"])
@pytest.mark.parametrize("mode,model", [("R", 0), ("P", 1)])
def test_hooks_field_streams(name, mode, model):
    """Field pictures and MBAFF frames through the hooks surface: the oracle's parser (field
    contexts, macroblock pairs) driven by the device's bins gives the pinned containers
    (tests/golden/fields.json) and the original file back."""
    g = {e["file"]: e for e in json.loads((ROOT / "tests/golden/fields.json").read_text())["files"]}[name]
    data = (FIX / name).read_bytes()
    r, avrc, walked = _call("hooks_compress", data, len(data), model)
    assert r == 0, r
    assert hashlib.sha256(avrc).hexdigest() == g[mode]["avrc_sha256"]
    r, back, walked_d = _call("hooks_decompress", avrc, len(avrc))
    assert r == 0, r
    assert walked_d == walked and back == data


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["paff_ipp.264", "mbaff_ib.264", "realshort.mp4"])
@pytest.mark.parametrize("mode,model", [("R", 0), ("P", 1), ("C", 3)])
def test_hooks_streaming_compress(name, mode, model):
    """A streaming session: the driver hands the file to avr_hooks_feed only as far as the slice it
    is about to decode (Annex-B: through that slice's NAL unit, in two pieces; MP4 with its moov
    box last: the whole file first, as a non-seekable mov demuxer reads it), each init_decoder
    traces its slice alone, and avr_hooks_end returns the same pinned container as the whole-file
    session -- which the whole-file session then decompresses through the hooks."""
    if name.endswith(".264"):
        gold = {e["file"]: e for e in json.loads((ROOT / "tests/golden/fields.json").read_text())["files"]}[name][mode]
    else:
        gold = GOLD[(name, mode)]
    data = (FIX / name).read_bytes()
    r, avrc, walked = _call("hooks_compress_stream", data, len(data), model)
    assert r == 0, r
    assert hashlib.sha256(avrc).hexdigest() == gold["avrc_sha256"]
    r, back, walked_d = _call("hooks_decompress", avrc, len(avrc))
    assert r == 0, r
    assert walked_d == walked > 0 and back == data


@pytest.mark.gpu
def test_hooks_detect_a_diverging_caller():
    """A container whose re-coded stream was altered: the device decompress either fails or
    yields different bins; either way the session must not report success with wrong bytes."""
    data = (FIX / "realshort.mp4").read_bytes()
    r, avrc, _ = _call("hooks_compress", data, len(data), 1)
    assert r == 0
    bad = bytearray(avrc)
    bad[len(bad) // 2] ^= 0x5A
    r, back, _ = _call("hooks_decompress", bytes(bad), len(bad))
    assert r != 0 or back != data or bytes(bad) == avrc


@pytest.mark.gpu
@pytest.mark.parametrize("mode,k,what", [
    (1, 5, "begin_coding_type(SIG_MAP) one bin late"),
    (2, 3, "frame_num repeated across two pictures"),
    (3, 40, "mb_xy off by one macroblock"),
    (4, 7, "begin_sub_mb with another scan8 index"),
])
def test_hooks_reject_misplaced_model_events(mode, k, what):
    """The model keys depend on where the caller places its model events (recode.cpp:166-207,
    824-843, 951-974): a caller that differs from the device's parse in ONE of them -- %s -- would
    get a container the reference would not write for it, so the session fails with
    AVR_ERR_FORMAT instead of returning the device's container."""
    L, _ = _driver()
    L.hooks_set_perturb.argtypes = [ctypes.c_int, ctypes.c_int]
    data = (FIX / "realshort.mp4").read_bytes()
    try:
        L.hooks_set_perturb(mode, k)
        r, _, _ = _call("hooks_compress", data, len(data), 1)
    finally:
        L.hooks_set_perturb(0, 0)
    assert r == -3, (what, r)
    r, avrc, _ = _call("hooks_compress", data, len(data), 1)   # unperturbed: accepted
    assert r == 0 and hashlib.sha256(avrc).hexdigest() == GOLD[("realshort.mp4", "P")]["avrc_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,model", [("R", 0), ("P", 1)])
def test_hooks_accept_slice_header_frame_num(mode, model):
    """A caller that passes frame_spec the slice header's frame_num, as the fork does: cockatoo.mp4
    has B pictures with nal_ref_idc 0, after which two consecutive pictures share frame_num (B 4, P 4;
    B 5, P 5; ...).  The session accepts that repeat (the device's pictures still turn the model's
    frames over) and gives the pinned container; a repeat where the headers' frame_num
    differ stays refused (test_hooks_reject_misplaced_model_events, perturbation 2)."""
    L, _ = _driver()
    L.hooks_set_frame_num_syntax.argtypes = [ctypes.c_int]
    data = (FIX / "cockatoo.mp4").read_bytes()
    try:
        L.hooks_set_frame_num_syntax(1)
        r, avrc, walked = _call("hooks_compress", data, len(data), model)
    finally:
        L.hooks_set_frame_num_syntax(0)
    assert r == 0, r
    assert hashlib.sha256(avrc).hexdigest() == GOLD[("cockatoo.mp4", mode)]["avrc_sha256"]


def _stream_with(fn, data, model, chunk):
    L, _ = _driver()
    L.hooks_set_feed_chunk.argtypes = [ctypes.c_size_t]
    try:
        L.hooks_set_feed_chunk(chunk)
        return _call(fn, data, len(data), model)
    finally:
        L.hooks_set_feed_chunk(0)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [4096, 32768])
@pytest.mark.parametrize("name", ["paff_ipp.264", "mbaff_ib.264", "realshort_faststart.mp4"])
def test_hooks_streaming_fixed_size_reads(name, chunk):
    """A streaming session fed in fixed-size reads (read_packet's buffer, not NAL boundaries), for
    Annex-B streams and a moov-first MP4 (its samples stream after the moov box): the
    container equals the oracle's for the same file, parallel model."""
    import tempfile
    from pathlib import Path
    from _oracle import oracle_cli
    from test_stream_ingest import INPUTS
    data = INPUTS[name]
    r, avrc, walked = _stream_with("hooks_compress_stream", data, 1, chunk)
    assert r == 0, r
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / name
        f.write_bytes(data)
        assert avrc == oracle_cli("compress", f, mode="P")
    r, back, walked_d = _call("hooks_decompress", avrc, len(avrc))
    assert r == 0 and back == data and walked_d == walked > 0


@pytest.mark.gpu
def test_hooks_streaming_1000_slices_flat():
    """1,000 slices (a tiled IP stream of small pictures, Annex-B) through a streaming session fed
    NAL unit by NAL unit: each init_decoder parses only the new unit and traces (and, parallel
    model, codes) only the new slice, so the per-slice host time stays flat -- the median of the
    last 100 slices within 1.5x of the first 100 (the whole-prefix re-parse grew linearly) -- and
    the container equals the oracle's."""
    import statistics
    import tempfile
    from pathlib import Path

    import avrecode_amd as avr
    from _oracle import oracle_cli
    with avr.Context(0) as ctx:
        data = ctx.synthesize(avr.SynthParams(mb_width=12, mb_height=8, slice_type=0, slice_qp=28, seed=77,
                                              gop_length=25, repeat=40), 25)
    assert len(avr.parse_stream(data).descs) == 1000
    r, avrc, walked = _stream_with("hooks_compress_stream", data, 1, 0)
    assert r == 0 and walked == 1000, (r, walked)
    L, _ = _driver()
    L.hooks_slice_times.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    buf = (ctypes.c_double * 1000)()
    assert L.hooks_slice_times(buf, 1000) == 1000
    t = list(buf)
    first, last = statistics.median(t[:100]), statistics.median(t[-100:])
    assert last <= 1.5 * first, (first, last)
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "s.264"
        f.write_bytes(data)
        assert avrc == oracle_cli("compress", f, mode="P")
