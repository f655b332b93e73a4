"""Test-side access to the oracle (oracle/, CPU restatement of the reference path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes
import os
import subprocess
import tempfile
from functools import lru_cache
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
ORACLE = ROOT / "oracle"


def build_oracle():
    lib, cli = ORACLE / "liboracle.so", ORACLE / "recode_oracle"
    if not lib.exists() or not cli.exists():
        subprocess.run(["make", "-s", "-C", str(ORACLE), "all"], check=True)
    return lib, cli


@lru_cache(None)
def lib():
    path, _ = build_oracle()
    L = ctypes.CDLL(str(path))
    L.avr_script_run.restype = ctypes.c_long
    L.avr_script_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    L.avr_script_decode_recoded.restype = ctypes.c_long
    L.avr_script_decode_recoded.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    L.avr_script_decode_cabac.restype = ctypes.c_long
    L.avr_script_decode_cabac.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    L.avr_script_decode_p.restype = ctypes.c_long
    L.avr_script_decode_p.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    return L


def _ops_array(ops):
    flat = []
    for op in ops:
        flat += [ord(op[0]), int(op[1]), int(op[2]), int(op[3])]
    return (ctypes.c_int32 * max(1, len(flat)))(*flat)


def script_encode(kind, ops):
    """kind: 'recoded', 'cabac' or 'p' (the P-format coder); ops: list of (op, a, b, c).  Returns bytes."""
    arr = _ops_array(ops)
    cap = 64 + 4 * len(ops)
    buf = ctypes.create_string_buffer(cap)
    n = lib().avr_script_run({"recoded": 0, "cabac": 1, "p": 2}[kind], arr, len(ops), buf, cap)
    assert n >= 0
    return buf.raw[:n]


def script_decode_ok(kind, data, ops):
    arr = _ops_array(ops)
    fn = {"recoded": lib().avr_script_decode_recoded, "cabac": lib().avr_script_decode_cabac,
          "p": lib().avr_script_decode_p}[kind]
    return fn(data, len(data), arr, len(ops))


@lru_cache(None)
def lps_table():
    """FFmpeg-layout rangeTabLPS (512 bytes) as the oracle builds it."""
    L = lib()
    return list((ctypes.c_uint8 * 512).in_dll(L, "avr_lps_range"))


def oracle_cli(cmd, path, mode="R", out=None, split_bytes=None):
    """Run recode_oracle; returns stdout bytes (or the output file's bytes).  split_bytes: the parallel
    model's long-slice split for this run (AVR_SPLIT_BYTES; None: the environment's / the default)."""
    _, cli = build_oracle()
    env = dict(os.environ)
    if split_bytes is not None:
        env["AVR_SPLIT_BYTES"] = str(int(split_bytes))
    with tempfile.TemporaryDirectory() as td:
        o = Path(td) / "out.bin"
        args = [str(cli), cmd] + {"R": [], "P": ["-p"], "P32": ["-p32"], "C": ["-c"]}[mode] + [str(path), str(o)]
        r = subprocess.run(args, capture_output=True, env=env)
        if r.returncode != 0:
            raise RuntimeError(f"recode_oracle {cmd} failed: {r.stderr.decode()}")
        if cmd == "roundtrip":
            return r.stdout
        return o.read_bytes()


def slices_p(data: bytes, lo: int = 0, hi: int = 1 << 62, check_recodable: bool = True, p32: bool = False):
    """Per-slice fresh-model (P-mode) compress -> decompress through the oracle, on the reference's
    arithmetic_code<uint64_t, uint8_t> (p32 False, MODEL_PARALLEL) or the P32 coder (MODEL_PARALLEL32).

    Returns (total_slices, records); each record is a dict with recodable, status_c, bins, recoded,
    status_d, regen (avr_oracle_slices_p, oracle/oracle_recode.c)."""
    import struct
    L = lib()
    f = L.avr_oracle_slices_p
    f.restype = ctypes.c_long
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_long, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
    out, olen = ctypes.c_void_p(), ctypes.c_size_t()
    total = f(data, len(data), lo, hi, 1 if check_recodable else 0, 1 if p32 else 0, ctypes.byref(out),
              ctypes.byref(olen))
    if total < 0:
        raise RuntimeError("avr_oracle_slices_p: demux failed")
    raw = ctypes.string_at(out.value, olen.value) if olen.value else b""
    ctypes.CDLL(None).free(ctypes.c_void_p(out.value))
    recs, p = [], 0
    while p < len(raw):
        rec, sc, bins, lc = struct.unpack_from("<iiII", raw, p)
        p += 16
        rc = raw[p:p + lc]
        p += lc
        sd, ld = struct.unpack_from("<iI", raw, p)
        p += 8
        rg = raw[p:p + ld]
        p += ld
        recs.append(dict(recodable=rec, status_c=sc, bins=bins, recoded=rc, status_d=sd, regen=rg))
    return total, recs


def patch_restores(regen: bytes, payload: bytes) -> bool:
    """decompressor::run's last-byte rule (recode.cpp:1345-1356) applied to regen equals payload."""
    size = len(payload)
    if size < 1:
        return False
    if (len(regen) & 1) != (size & 1):
        fixed = regen + payload[-1:]
    else:
        fixed = regen[:-1] + payload[-1:] if regen else b""
    return fixed == payload
