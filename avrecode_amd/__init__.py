"""avrecode-amd: MI355X-native CABAC recode path (ddkang/avrecode's decode -> predict -> re-encode).

Python view of the C ABI in include/avrecode.h (libavrecode.so, built in-tree by
``make -C avrecode_amd``).  The product is the native library and the ``recode`` CLI next to it;
this module is the binding tests, bench.py and the sharded driver use.  There is no Python or CPU
implementation of the hot path: without the library, or without a GPU, every call raises.

Reference interfaces mirrored here (file:line in ddkang/avrecode):
  compress / decompress / roundtrip   recode.cpp:1102-1125, 1312-1357, 1594-1624 (+ CLI 1626-1660)
  parse_stream                        av_decoder::decode_video -> init_decoder(buf, size), recode.cpp:73-143
  Context.compress_slices / ...       compressor::cabac_decoder / decompressor::cabac_decoder per
                                      slice, recode.cpp:1134-1268, 1411-1520
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

__all__ = [
    "AvrError", "Context", "MODEL_REFERENCE", "MODEL_PARALLEL", "MODEL_PARALLEL32", "MODEL_CHAINED", "MODEL_NAMES",
    "SLICE_DESC",
    "SLICE_RESULT", "SynthParams", "lib", "parse_stream", "assemble_container", "neighbor_tables",
    "plan_decompress", "splice_container", "container_model", "source_sha", "library_path", "EXPORTED_SYMBOLS",
    "seams_of_container",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# AVR_LIBRARY selects an instrumented build (e.g. prof/libavrecode.so, `make -C avrecode_amd prof`)
library_path = os.environ.get("AVR_LIBRARY") or os.path.join(_HERE, "libavrecode.so")

# avr_model (include/avrecode.h): the reference model; the parallel model (fresh model per slice)
# on the reference's arithmetic_code<uint64_t, uint8_t>; the parallel model on the optional P32 coder
MODEL_REFERENCE = 0
MODEL_PARALLEL = 1
MODEL_PARALLEL32 = 2
MODEL_CHAINED = 3   # the reference model in chains of CHAIN_SLICES coded slices ("avrecode-amd:R16")
CHAIN_SLICES = 16
SPLIT_BYTES_DEFAULT = 98304   # the parallel model's long-slice split (Context.split_bytes), unless AVR_SPLIT_BYTES
MODEL_NAMES = {MODEL_REFERENCE: "R", MODEL_PARALLEL: "P", MODEL_PARALLEL32: "P32", MODEL_CHAINED: "C"}

AVR_OK = 0
_STATUS = {
    -1: "invalid argument", -2: "device error", -3: "format error", -4: "out of memory",
    -5: "roundtrip mismatch", -6: "unsupported",
}

# every function include/avrecode.h declares
EXPORTED_SYMBOLS = (
    "avr_create", "avr_destroy", "avr_last_error", "avr_free", "avr_compress_file", "avr_decompress_file",
    "avr_roundtrip_file", "avr_compress_slices", "avr_decompress_slices", "avr_pack_outputs",
    "avr_roundtrip_slices", "avr_derive_decompress_descs", "avr_verify_slices", "avr_parse_stream",
    "avr_assemble_container", "avr_assemble_container_parsed", "avr_assemble_container_into", "avr_parse_stream_range", "avr_slice_payload_sizes", "avr_dec_plan_new", "avr_dec_plan_free", "avr_dec_plan_load", "avr_dec_plan_descs", "avr_dec_plan_arena", "avr_dec_plan_splice", "avr_container_model", "avr_synthesize_stream",
    "avr_container_describe", "avr_compress_files", "avr_decompress_files",
    "avr_hooks_compress_begin", "avr_hooks_compress_stream_begin", "avr_hooks_feed",
    "avr_hooks_decompress_begin", "avr_hook_init_decoder", "avr_hook_get",
    "avr_hook_get_bypass", "avr_hook_get_terminate", "avr_hook_skip_bytes", "avr_hook_frame_spec", "avr_hook_mb_xy",
    "avr_hook_begin_sub_mb", "avr_hook_end_sub_mb", "avr_hook_begin_coding_type", "avr_hook_end_coding_type",
    "avr_hooks_end", "avr_hooks_destroy", "avr_neighbor_tables", "avr_last_phase_times",
    "avr_plan_decompress", "avr_splice_container", "avr_roundtrip_files", "avr_slice_kernel",
    "avr_compress_chain_range", "avr_decompress_chain_range", "avr_set_split_bytes", "avr_get_split_bytes",
)

# avr_slice_desc / avr_slice_result (include/avrecode.h), C layout
SLICE_DESC = np.dtype([
    ("payload_offset", "<u8"), ("payload_size", "<u4"), ("read_limit", "<u4"),
    ("out_offset", "<u8"), ("out_capacity", "<u4"),
    ("slice_type", "<i4"), ("slice_qp", "<i4"), ("cabac_init_idc", "<i4"), ("first_mb", "<i4"),
    ("mb_width", "<i4"), ("mb_height", "<i4"), ("num_ref_idx_l0", "<i4"), ("num_ref_idx_l1", "<i4"),
    ("chroma_array_type", "<i4"), ("transform_8x8_mode", "<i4"), ("direct_8x8_inference", "<i4"),
    ("x264_build", "<i4"), ("picture_id", "<i4"), ("coded", "<i4"), ("structure", "<i4"),
    ("file_offset", "<u8"),
], align=True)
SLICE_RESULT = np.dtype([("out_len", "<u4"), ("status", "<i4"), ("bins", "<u4"), ("mbs", "<u4"),
                         ("bill", "<u4", (6,))], align=True)
# avr_pip_coding_type (CodingType, recode.cpp:616): the index of avr_file_stats.bill / cabac_bill
CODING_TYPES = ("PIP_UNKNOWN", "PIP_UNREACHABLE", "PIP_SIGNIFICANCE_MAP", "PIP_SIGNIFICANCE_EOB",
                "PIP_SIGNIFICANCE_NZ", "PIP_RESIDUALS")
assert SLICE_DESC.itemsize == 96 and SLICE_RESULT.itemsize == 40


class AvrError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"avrecode: {_STATUS.get(code, code)}: {msg}")
        self.code = code


PHASES = ("demux_s", "upload_s", "kernel_s", "download_s", "container_s", "other_s")


class _PhaseTimes(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in PHASES]


def _phases(p: _PhaseTimes) -> dict:
    return {n: getattr(p, n) for n in PHASES}


class _FileStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("file_bytes", "slices", "coded_slices", "skipped_slices", "payload_bytes", "recoded_bytes", "bins")] + \
               [("compress_s", ctypes.c_double), ("decompress_s", ctypes.c_double),
                ("bill", ctypes.c_uint64 * 6), ("cabac_bill", ctypes.c_uint64 * 6),
                ("attempts", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("compress_phases", _PhaseTimes), ("decompress_phases", _PhaseTimes)]


class _SynthParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("mb_width", "mb_height", "slice_type", "slice_qp", "chroma_format_idc", "transform_8x8_mode",
                 "num_ref_idx_l0", "num_ref_idx_l1")] + [("seed", ctypes.c_uint64)] + \
               [("slices_per_picture", ctypes.c_int32), ("gop_length", ctypes.c_int32), ("repeat", ctypes.c_int32),
                ("structure", ctypes.c_int32)]


@dataclass
class SynthParams:
    """Synthetic slice parameters (avr_synth_params); defaults = one 1080p 4:2:0 High I picture."""
    mb_width: int = 120
    mb_height: int = 68
    slice_type: int = 2
    slice_qp: int = 26
    chroma_format_idc: int = 1
    transform_8x8_mode: int = 1
    num_ref_idx_l0: int = 1
    num_ref_idx_l1: int = 1
    seed: int = 0
    slices_per_picture: int = 1
    gop_length: int = 0          # > 0: IDR I picture every gop_length pictures, slice_type between
    repeat: int = 1              # > 1: the pictures written this many times (frame numbers advance)
    structure: int = 0           # 0 progressive, 1 field pictures (PAFF), 2 MBAFF frames, 3 PAFF bottom first


_lib = None


def source_sha() -> str:
    """sha256 over the native sources libavrecode.so is built from (avrecode_amd/csrc/*,
    include/avrecode.h, the Makefile): identifies the build a profile was taken on, without git
    (the GPU box has no .git).  scripts/pmc_traffic.py records it; bench.py uses a traffic
    profile only when it matches the tree being measured."""
    import hashlib
    root = os.path.dirname(_HERE)
    files = sorted(os.path.join(_HERE, "csrc", f) for f in os.listdir(os.path.join(_HERE, "csrc")))
    files += [os.path.join(root, "include", "avrecode.h"), os.path.join(_HERE, "Makefile")]
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def lib() -> ctypes.CDLL:
    """Load libavrecode.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(library_path):
        raise ImportError(f"{library_path} is missing: build it with `make -C {_HERE}` (or __graft_entry__.build())")
    L = ctypes.CDLL(library_path)
    vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    pp = ctypes.POINTER(ctypes.c_void_p)
    psz = ctypes.POINTER(ctypes.c_size_t)
    pi = ctypes.POINTER(ctypes.c_int)
    L.avr_create.argtypes = [i32, pp]
    L.avr_destroy.argtypes = [vp]
    L.avr_destroy.restype = None
    L.avr_last_error.argtypes = [vp]
    L.avr_last_error.restype = ctypes.c_char_p
    L.avr_free.argtypes = [vp]
    L.avr_free.restype = None
    L.avr_compress_file.argtypes = [vp, vp, sz, i32, pp, psz]
    L.avr_decompress_file.argtypes = [vp, vp, sz, pp, psz]
    L.avr_roundtrip_file.argtypes = [vp, vp, sz, i32, pp, psz, ctypes.POINTER(_FileStats)]
    for f in (L.avr_compress_slices, L.avr_decompress_slices):
        f.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, i32, vp]
    L.avr_roundtrip_slices.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, i32, vp]
    L.avr_derive_decompress_descs.argtypes = [vp, vp, vp, i32, vp, vp]
    L.avr_verify_slices.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp]
    L.avr_slice_kernel.argtypes = [vp, i32, i32, i32, ctypes.POINTER(ctypes.c_int)]
    L.avr_compress_chain_range.argtypes = [vp, vp, sz, i32, i32] + [vp] * 7
    L.avr_decompress_chain_range.argtypes = [vp, vp, sz, i32, i32] + [vp] * 7
    L.avr_pack_outputs.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp]
    L.avr_parse_stream.argtypes = [vp, sz, pp, pi, pp, psz, psz, pi, pi]
    L.avr_parse_stream_range.argtypes = [vp, sz, i32, i32, pp, pi, pp, psz, psz, pi, pi]
    L.avr_slice_payload_sizes.argtypes = [vp, sz, pp, pi]
    L.avr_assemble_container.argtypes = [vp, sz, i32, i32, vp, vp, sz, vp, vp, pp, psz]
    L.avr_assemble_container_parsed.argtypes = [vp, sz, i32, vp, i32, vp, sz, vp, vp, sz, vp, vp, pp, psz]
    L.avr_assemble_container_into.argtypes = [vp, sz, i32, vp, i32, vp, sz, vp, vp, sz, vp, vp, vp, sz, psz]
    L.avr_dec_plan_new.argtypes = [pp]
    L.avr_dec_plan_free.argtypes = [vp]
    L.avr_dec_plan_free.restype = None
    L.avr_dec_plan_load.argtypes = [vp, vp, sz, pi, psz, psz, pi, pi]
    L.avr_dec_plan_descs.argtypes = [vp, vp]
    L.avr_dec_plan_arena.argtypes = [vp, vp, sz]
    L.avr_dec_plan_splice.argtypes = [vp, vp, vp, sz, vp, vp, vp, sz, psz]
    L.avr_container_model.argtypes = [vp, sz, pi]
    L.avr_synthesize_stream.argtypes = [vp, ctypes.POINTER(_SynthParams), i32, pp, psz]
    L.avr_container_describe.argtypes = [vp, sz, pp, pp, psz]
    L.avr_compress_files.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp]
    L.avr_decompress_files.argtypes = [vp, i32, vp, vp, vp, vp, vp]
    L.avr_roundtrip_files.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp, vp]
    L.avr_neighbor_tables.argtypes = [vp, vp]
    L.avr_plan_decompress.argtypes = [vp, sz, pp, pi, pp, psz, psz, pi, pi]
    L.avr_splice_container.argtypes = [vp, sz, i32, vp, vp, sz, vp, vp, pp, psz]
    L.avr_last_phase_times.argtypes = [vp, vp]
    L.avr_set_split_bytes.argtypes = [vp, sz]
    L.avr_get_split_bytes.argtypes = [vp]
    L.avr_get_split_bytes.restype = sz
    for name in EXPORTED_SYMBOLS:   # fails here, not at first use, when the build is stale
        getattr(L, name)
    _lib = L
    return L


def _buf(data) -> tuple[ctypes.c_void_p, int, object]:
    """(pointer, length, keepalive) for bytes / bytearray / memoryview / numpy uint8, without a copy
    (the library only reads its inputs; a 4.47 GB stream must not be duplicated per call)."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).reshape(-1).view(np.uint8)
    elif isinstance(data, (bytes, bytearray, memoryview)):
        a = np.frombuffer(data, dtype=np.uint8)
    else:
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    if a.nbytes == 0:   # a valid, non-null pointer for empty inputs
        cb = ctypes.create_string_buffer(1)
        return ctypes.cast(cb, ctypes.c_void_p), 0, cb
    return ctypes.c_void_p(a.ctypes.data), a.nbytes, a


def _take(p: ctypes.c_void_p, n: int) -> bytes:
    L = lib()
    try:
        if not n:
            return b""
        # ctypes.string_at's length is a C int: a buffer of 2 GiB or more (a 10-minute 4K stream,
        # its container) is copied through an array view instead
        return ctypes.string_at(p.value, n) if n < (1 << 31) else bytes((ctypes.c_char * n).from_address(p.value))
    finally:
        L.avr_free(p)


class _LibBuffer:
    """A malloc'd library buffer exposed to numpy without a copy; freed (avr_free) when the last
    array viewing it is gone (numpy keeps this object as every view's base)."""

    def __init__(self, p: int, n: int):
        self._p = p
        self._free = lib().avr_free   # held: at interpreter exit the module's globals may be gone
        self._vp = ctypes.c_void_p
        self.__array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (p, False), "version": 3}

    def __del__(self):
        if self._p:
            self._free(self._vp(self._p))
            self._p = 0


def _take_array(p: ctypes.c_void_p, n: int) -> np.ndarray:
    """A library buffer as a numpy uint8 array, without copying it (a 4 GB parse or container is not
    copied again); the buffer is freed with the array."""
    if not n or not p.value:
        if p.value:
            lib().avr_free(p)
        return np.zeros(0, dtype=np.uint8)
    return np.asarray(_LibBuffer(p.value, n))


@dataclass
class ParsedStream:
    """Per-slice descriptors + payload arena (what init_decoder receives, recode.cpp:143)."""
    descs: np.ndarray        # SLICE_DESC[n]
    arena: np.ndarray        # uint8 payloads (16-byte aligned, zero padded)
    work_len: int            # bytes of compress output space the descs' out_offset/out_capacity index
    max_mb_width: int
    max_mb_height: int

    @property
    def payload_bytes(self) -> int:
        return int(self.descs["payload_size"].sum())


def parse_stream(data, lo: int = 0, hi: "int | None" = None) -> ParsedStream:
    """Host-side slice extraction (avr_parse_stream; with a slice range [lo, hi),
    avr_parse_stream_range: that range only, rebased as shard.subset would).  Needs no GPU."""
    L = lib()
    p, n, keep = _buf(data)
    descs, arena = ctypes.c_void_p(), ctypes.c_void_p()
    ns, mw, mh = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    alen, wlen = ctypes.c_size_t(), ctypes.c_size_t()
    if lo == 0 and hi is None:
        r = L.avr_parse_stream(p, n, ctypes.byref(descs), ctypes.byref(ns), ctypes.byref(arena), ctypes.byref(alen),
                               ctypes.byref(wlen), ctypes.byref(mw), ctypes.byref(mh))
    else:
        r = L.avr_parse_stream_range(p, n, int(lo), -1 if hi is None else int(hi), ctypes.byref(descs),
                                     ctypes.byref(ns), ctypes.byref(arena), ctypes.byref(alen), ctypes.byref(wlen),
                                     ctypes.byref(mw), ctypes.byref(mh))
    del keep
    if r != AVR_OK:
        raise AvrError(r, "avr_parse_stream failed")
    d = _take_array(descs, ns.value * SLICE_DESC.itemsize).view(SLICE_DESC)
    a = _take_array(arena, alen.value)
    return ParsedStream(d, a, int(wlen.value), int(mw.value), int(mh.value))


def slice_payload_sizes(data) -> np.ndarray:
    """Every CABAC slice's payload_size (avr_slice_payload_sizes): a sharded run's partition input,
    without copying the payloads.  Host only."""
    p, n, keep = _buf(data)
    out, ns = ctypes.c_void_p(), ctypes.c_int()
    r = lib().avr_slice_payload_sizes(p, n, ctypes.byref(out), ctypes.byref(ns))
    if r != AVR_OK:
        raise AvrError(r, "avr_slice_payload_sizes failed")
    return _take_array(out, 4 * ns.value).view(np.uint32)


def plan_decompress(avrc) -> ParsedStream:
    """A PARALLEL-model container's coded slices as a decompress batch (avr_plan_decompress): the
    descs' payloads are the re-coded streams, their outputs the regenerated CABAC bytes.  Host only."""
    L = lib()
    p, n, keep = _buf(avrc)
    descs, arena = ctypes.c_void_p(), ctypes.c_void_p()
    ns, mw, mh = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    alen, wlen = ctypes.c_size_t(), ctypes.c_size_t()
    r = L.avr_plan_decompress(p, n, ctypes.byref(descs), ctypes.byref(ns), ctypes.byref(arena), ctypes.byref(alen),
                              ctypes.byref(wlen), ctypes.byref(mw), ctypes.byref(mh))
    del keep
    if r != AVR_OK:
        raise AvrError(r, "avr_plan_decompress failed")
    d = _take_array(descs, ns.value * SLICE_DESC.itemsize).view(SLICE_DESC)
    a = _take_array(arena, alen.value)
    return ParsedStream(d, a, int(wlen.value), int(mw.value), int(mh.value))


class DecompressPlan:
    """The sharded decompress's host halves on one parse of a PARALLEL-model container
    (avr_dec_plan_*): load(avrc) plans it (no bytes copied), parsed(arena_out) gives the decompress
    batch (descs + the re-coded streams' arena, written into arena_out when given), splice(...) the
    file from the regenerated slices (into out when given: the view holding the file is returned).
    The handle keeps its scratch across loads; the container passed to load must stay alive and
    unchanged until the next load.  Host only."""

    def __init__(self):
        self._h = ctypes.c_void_p()
        r = lib().avr_dec_plan_new(ctypes.byref(self._h))
        if r != AVR_OK:
            raise AvrError(r, "avr_dec_plan_new failed")
        self._keep = None

    def load(self, avrc) -> "DecompressPlan":
        p, n, keep = _buf(avrc)
        ns, mw, mh = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        al, wl = ctypes.c_size_t(), ctypes.c_size_t()
        r = lib().avr_dec_plan_load(self._h, p, n, ctypes.byref(ns), ctypes.byref(al), ctypes.byref(wl),
                                    ctypes.byref(mw), ctypes.byref(mh))
        if r != AVR_OK:
            self._keep = None
            raise AvrError(r, "avr_dec_plan_load failed")
        self._keep = (avrc, keep)
        self.n_slices, self.arena_len, self.work_len = ns.value, al.value, wl.value
        self.max_mb_width, self.max_mb_height = mw.value, mh.value
        d = np.zeros(self.n_slices, dtype=SLICE_DESC)
        if self.n_slices:
            lib().avr_dec_plan_descs(self._h, d.ctypes.data)
        self.descs = d
        return self

    def parsed(self, arena_out: "np.ndarray | None" = None) -> ParsedStream:
        a = np.empty(self.arena_len, dtype=np.uint8) if arena_out is None else arena_out[:self.arena_len]
        if a.nbytes < self.arena_len:
            raise ValueError("DecompressPlan.parsed: arena_out too small")
        r = lib().avr_dec_plan_arena(self._h, a.ctypes.data, a.nbytes)
        if r != AVR_OK:
            raise AvrError(r, "avr_dec_plan_arena failed")
        return ParsedStream(self.descs.copy(), a, self.work_len, self.max_mb_width, self.max_mb_height)

    def splice(self, status, regen, offsets, lens, out: "np.ndarray | None" = None):
        st = np.ascontiguousarray(status, dtype=np.int32)
        of = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        if len(st) != self.n_slices or len(of) != len(st) or len(ln) != len(st):
            raise ValueError("DecompressPlan.splice: one status / offset / length per planned slice")
        rp, rn, keep = _buf(regen)
        olen = ctypes.c_size_t()
        L = lib()
        if out is None:
            L.avr_dec_plan_splice(self._h, st.ctypes.data, rp, rn, of.ctypes.data, ln.ctypes.data, None, 0,
                                  ctypes.byref(olen))
            out = np.empty(olen.value, dtype=np.uint8)
        r = L.avr_dec_plan_splice(self._h, st.ctypes.data, rp, rn, of.ctypes.data, ln.ctypes.data, out.ctypes.data,
                                  out.nbytes, ctypes.byref(olen))
        if r != AVR_OK:
            raise AvrError(r, f"avr_dec_plan_splice failed (file {olen.value} B, buffer {out.nbytes} B)")
        return out[:olen.value]

    def close(self):
        if self._h:
            lib().avr_dec_plan_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def container_model(avrc) -> int:
    """The model mode a Recoded container was written with (avr_container_model): MODEL_*.  Host only."""
    p, n, keep = _buf(avrc)
    m = ctypes.c_int()
    r = lib().avr_container_model(p, n, ctypes.byref(m))
    if r != AVR_OK:
        raise AvrError(r, "avr_container_model failed")
    return int(m.value)


def splice_container(avrc, status: np.ndarray, regen, offsets: np.ndarray, lens: np.ndarray) -> bytes:
    """The original file from a PARALLEL-model container and its slices' regenerated bytes
    (avr_splice_container; last-byte patch applied here).  regen: bytes or a uint8 array.  Host only."""
    L = lib()
    p, n, keep = _buf(avrc)
    st = np.ascontiguousarray(status, dtype=np.int32)
    of = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint32)
    rp, rn, keep2 = _buf(regen)
    out, olen = ctypes.c_void_p(), ctypes.c_size_t()
    r = L.avr_splice_container(p, n, len(st), st.ctypes.data, rp, rn, of.ctypes.data, ln.ctypes.data,
                               ctypes.byref(out), ctypes.byref(olen))
    if r != AVR_OK:
        raise AvrError(r, "avr_splice_container failed")
    return _take(out, olen.value)


def container_bound(n_file: int, n_slices: int, recoded_bytes: int) -> int:
    """An upper bound on the size of a container assembled from n_slices slices of a file of n_file
    bytes with recoded_bytes re-coded bytes in all (avr_assemble_container_into's buffer)."""
    return int(n_file) + int(recoded_bytes) + 64 * (int(n_slices) + 2)


def assemble_container(data, status: np.ndarray, recoded, offsets: np.ndarray, lens: np.ndarray,
                       model: int = MODEL_PARALLEL, ps: "ParsedStream | None" = None, as_array: bool = False,
                       out: "np.ndarray | None" = None):
    """Recoded container from per-slice outputs gathered from the ranks (avr_assemble_container; with ps =
    parse_stream(data) already in hand, avr_assemble_container_parsed: no second parse).  recoded:
    bytes or a uint8 array.  model: the model / coder the outputs were made with (PARALLEL, PARALLEL32,
    or CHAINED for Context.compress_chain_range's outputs).  as_array: the container
    as a uint8 array over the library's buffer (no copy into bytes).  out (with ps): a uint8 array
    the container is written into (avr_assemble_container_into; container_bound() bytes suffice);
    returns the view of it that holds the container.  Host only."""
    L = lib()
    p, n, keep = _buf(data)
    st = np.ascontiguousarray(status, dtype=np.int32)
    of = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint32)
    rp, rn, keep2 = _buf(recoded)
    res, olen = ctypes.c_void_p(), ctypes.c_size_t()
    if out is not None:
        if ps is None or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError("assemble_container: out needs ps and a contiguous uint8 array")
        dd = np.ascontiguousarray(ps.descs)
        if len(dd) != len(st) or len(of) != len(st) or len(ln) != len(st):
            raise ValueError("assemble_container: status / offsets / lens need one entry per parsed slice")
        r = L.avr_assemble_container_into(p, n, model, dd.ctypes.data, len(dd), ps.arena.ctypes.data, ps.arena.nbytes,
                                          st.ctypes.data, rp, rn, of.ctypes.data, ln.ctypes.data, out.ctypes.data,
                                          out.nbytes, ctypes.byref(olen))
        if r != AVR_OK:
            raise AvrError(r, f"avr_assemble_container_into failed (container {olen.value} B, buffer {out.nbytes} B)")
        return out[:olen.value]
    if ps is not None:
        dd = np.ascontiguousarray(ps.descs)
        if len(dd) != len(st) or len(of) != len(st) or len(ln) != len(st):
            raise ValueError("assemble_container: status / offsets / lens need one entry per parsed slice")
        r = L.avr_assemble_container_parsed(p, n, model, dd.ctypes.data, len(dd), ps.arena.ctypes.data, ps.arena.nbytes,
                                            st.ctypes.data, rp, rn, of.ctypes.data, ln.ctypes.data, ctypes.byref(res),
                                            ctypes.byref(olen))
    else:
        r = L.avr_assemble_container(p, n, model, len(st), st.ctypes.data, rp, rn, of.ctypes.data, ln.ctypes.data,
                                     ctypes.byref(res), ctypes.byref(olen))
    if r != AVR_OK:
        raise AvrError(r, "avr_assemble_container failed")
    return _take_array(res, olen.value) if as_array else _take(res, olen.value)


def _varint(b, i: int) -> tuple[int, int]:
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def seams_of_container(avrc) -> list:
    """The parallel model's long-slice split in a container: (block index, seams field bytes) of every
    coded block that was cut (Block field 16, include/avrecode.h avr_set_split_bytes).  A plain walk
    of the wire format (host only, no library call)."""
    b = memoryview(bytes(avrc))
    out, i, k = [], 0, 0
    while i < len(b):
        tag, i = _varint(b, i)
        wt = tag & 7
        if wt == 0:
            _, i = _varint(b, i)
            continue
        if wt != 2:
            raise ValueError("not a Recoded message")
        n, i = _varint(b, i)
        if tag >> 3 == 2:   # a Block: look for field 16
            j, e = i, i + n
            while j < e:
                t2, j = _varint(b, j)
                if t2 & 7 == 0:
                    _, j = _varint(b, j)
                    continue
                l2, j = _varint(b, j)
                if t2 >> 3 == 16:
                    out.append((k, l2))
                j += l2
            k += 1
        i += n
    return out


def describe_container(avrc) -> tuple[dict, bytes]:
    """Parse a Recoded protobuf with the library's wire codec (avr_container_describe): its fields
    (hex strings for bytes) and the message re-serialised by the library's writer.  Host only."""
    import json
    L = lib()
    p, n, keep = _buf(avrc)
    js, out, olen = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_size_t()
    r = L.avr_container_describe(p, n, ctypes.byref(js), ctypes.byref(out), ctypes.byref(olen))
    if r != AVR_OK:
        raise AvrError(r, "avr_container_describe failed")
    text = ctypes.string_at(js.value).decode()
    L.avr_free(js)
    return json.loads(text), _take(out, olen.value)


def neighbor_tables(ctx=None) -> tuple[bytes, bytes]:
    """(nb_left[48], nb_up[48]): the model's neighbour geometry as the kernels use it
    (avr_neighbor_tables).  ctx None: the host-built table (no GPU); a Context: its device copy."""
    L = lib()
    out = ctypes.create_string_buffer(96)
    r = L.avr_neighbor_tables(ctx._h if ctx is not None else None, out)
    if r != AVR_OK:
        raise AvrError(r, "avr_neighbor_tables failed")
    return out.raw[:48], out.raw[48:96]


class Context:
    """One device context (avr_ctx).  Raises AvrError(AVR_ERR_DEVICE) when no GPU is usable."""

    def __init__(self, device: int = 0):
        L = lib()
        h = ctypes.c_void_p()
        r = L.avr_create(int(device), ctypes.byref(h))
        if r != AVR_OK:
            raise AvrError(r, f"avr_create(device={device}) failed (no usable GPU? the hot path has no CPU path)")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().avr_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, r: int, what: str):
        if r != AVR_OK:
            raise AvrError(r, f"{what}: {lib().avr_last_error(self._h).decode(errors='replace')}")

    @property
    def split_bytes(self) -> int:
        """The parallel model's long-slice split (avr_set_split_bytes; 0: none): the whole-file
        compress cuts a progressive slice into pieces of about this many payload bytes."""
        return int(lib().avr_get_split_bytes(self._h))

    @split_bytes.setter
    def split_bytes(self, v: int):
        self._check(lib().avr_set_split_bytes(self._h, int(v)), "avr_set_split_bytes")

    # ------------------------------------------------------------------ whole files
    def compress(self, data, model: int = MODEL_REFERENCE) -> bytes:
        p, n, keep = _buf(data)
        out, olen = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(lib().avr_compress_file(self._h, p, n, model, ctypes.byref(out), ctypes.byref(olen)),
                    "compress")
        return _take(out, olen.value)

    def decompress(self, data) -> bytes:
        p, n, keep = _buf(data)
        out, olen = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(lib().avr_decompress_file(self._h, p, n, ctypes.byref(out), ctypes.byref(olen)), "decompress")
        return _take(out, olen.value)

    def roundtrip(self, data, model: int = MODEL_REFERENCE) -> tuple[bytes, dict]:
        p, n, keep = _buf(data)
        out, olen = ctypes.c_void_p(), ctypes.c_size_t()
        st = _FileStats()
        self._check(lib().avr_roundtrip_file(self._h, p, n, model, ctypes.byref(out), ctypes.byref(olen),
                                             ctypes.byref(st)), "roundtrip")
        stats = {f: getattr(st, f) for f, _ in _FileStats._fields_ if f != "reserved"}
        for f in ("compress_phases", "decompress_phases"):
            stats[f] = _phases(stats[f])
        for f in ("bill", "cabac_bill"):   # by CodingType name, nonzero entries (~h264_model's print)
            stats[f] = {CODING_TYPES[i]: int(v) for i, v in enumerate(stats[f]) if v}
        return _take(out, olen.value), stats

    def _files(self, fn, datas, *extra, tail=()):
        n = len(datas)
        keep = [_buf(d) for d in datas]
        ptrs = (ctypes.c_void_p * max(1, n))(*[k[0].value for k in keep])
        lens = (ctypes.c_size_t * max(1, n))(*[k[1] for k in keep])
        outs = (ctypes.c_void_p * max(1, n))()
        olens = (ctypes.c_size_t * max(1, n))()
        st = (ctypes.c_int32 * max(1, n))()
        self._check(fn(self._h, n, ptrs, lens, *extra, outs, olens, st, *tail), fn.__name__)
        res = []
        failed = [k for k in range(n) if st[k] != AVR_OK]
        # the context keeps one error message: it belongs to a failed file only when there is one
        detail = lib().avr_last_error(self._h).decode(errors="replace") if len(failed) == 1 else ""
        for k in range(n):
            if st[k] != AVR_OK:
                res.append(AvrError(st[k], f"file {k}" + (f": {detail}" if detail else "")))
            else:
                res.append(_take(ctypes.c_void_p(outs[k]), olens[k]))
        del keep
        return res

    def last_phase_times(self) -> dict:
        """avr_last_phase_times: where the last whole-file call's wall time went (seconds)."""
        p = _PhaseTimes()
        self._check(lib().avr_last_phase_times(self._h, ctypes.byref(p)), "avr_last_phase_times")
        return _phases(p)

    def compress_files(self, datas, model: int = MODEL_REFERENCE) -> list:
        """avr_compress_files: one container (bytes) or AvrError per input file."""
        return self._files(lib().avr_compress_files, datas, model)

    def decompress_files(self, datas) -> list:
        """avr_decompress_files: the original file (bytes) or AvrError per container."""
        return self._files(lib().avr_decompress_files, datas)

    def roundtrip_files(self, datas, model: int = MODEL_REFERENCE) -> tuple[list, dict]:
        """avr_roundtrip_files: (one container (bytes) or AvrError per input file, {"compress_s",
        "decompress_s"}: wall seconds of the batched compress and decompress calls)."""
        times = (ctypes.c_double * 2)()
        res = self._files(lib().avr_roundtrip_files, datas, model, tail=(times,))
        return res, {"compress_s": times[0], "decompress_s": times[1]}

    # ------------------------------------------------------- device-resident slice batches
    # All tensor arguments are torch tensors on this context's device (uint8 buffers, and uint8
    # views of descriptor/result arrays); `stream` is a torch.cuda.Stream or None (= its current).
    @staticmethod
    def _ptr(t) -> ctypes.c_void_p:
        return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p()

    @staticmethod
    def _stream(stream):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        return ctypes.c_void_p(s.cuda_stream)

    def compress_slices(self, d_desc, n, max_w, max_h, d_in, d_out, d_res, model=MODEL_PARALLEL, stream=None):
        self._check(lib().avr_compress_slices(self._h, self._ptr(d_desc), n, max_w, max_h, self._ptr(d_in),
                                              self._ptr(d_out), self._ptr(d_res), model, self._stream(stream)),
                    "compress_slices")

    def decompress_slices(self, d_desc, n, max_w, max_h, d_in, d_out, d_res, model=MODEL_PARALLEL, stream=None):
        self._check(lib().avr_decompress_slices(self._h, self._ptr(d_desc), n, max_w, max_h, self._ptr(d_in),
                                                self._ptr(d_out), self._ptr(d_res), model, self._stream(stream)),
                    "decompress_slices")

    def roundtrip_slices(self, d_desc, n, max_w, max_h, d_in, d_work, d_regen, d_dec_desc, d_res_c, d_res_d,
                         d_verdict, model=MODEL_PARALLEL, stream=None):
        P = self._ptr
        self._check(lib().avr_roundtrip_slices(self._h, P(d_desc), n, max_w, max_h, P(d_in), P(d_work), P(d_regen),
                                               P(d_dec_desc), P(d_res_c), P(d_res_d), P(d_verdict), model,
                                               self._stream(stream)), "roundtrip_slices")

    def derive_decompress_descs(self, d_desc, d_res_c, n, d_dec_desc, stream=None):
        P = self._ptr
        self._check(lib().avr_derive_decompress_descs(self._h, P(d_desc), P(d_res_c), n, P(d_dec_desc),
                                                      self._stream(stream)), "derive_decompress_descs")

    def verify_slices(self, d_desc, d_res_c, d_res_d, n, d_in, d_regen, d_verdict, stream=None):
        P = self._ptr
        self._check(lib().avr_verify_slices(self._h, P(d_desc), P(d_res_c), P(d_res_d), n, P(d_in), P(d_regen),
                                            P(d_verdict), self._stream(stream)), "verify_slices")

    def _chain_range(self, fn, name, data, world: int, rank: int):
        p, n, keep = _buf(data)
        lo, hi = ctypes.c_int(), ctypes.c_int()
        st, blob, offs, lens = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        blen = ctypes.c_size_t()
        r = fn(self._h, p, n, world, rank, ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(st), ctypes.byref(blob),
               ctypes.byref(blen), ctypes.byref(offs), ctypes.byref(lens))
        del keep
        self._check(r, name)
        k = hi.value - lo.value
        return (lo.value, hi.value, _take_array(st, 4 * k).view(np.int32), _take_array(blob, blen.value),
                _take_array(offs, 8 * k).view(np.uint64), _take_array(lens, 4 * k).view(np.uint32))

    def compress_chain_range(self, data, world: int, rank: int):
        """This rank's chains of a chained-model compress of one file (avr_compress_chain_range):
        (lo, hi, status int32, recoded uint8, offsets uint64, lens uint32) for the file's slices
        [lo, hi); status 0 coded, -1 not coded, -2 failed (compress the file whole)."""
        return self._chain_range(lib().avr_compress_chain_range, "compress_chain_range", data, world, rank)

    def decompress_chain_range(self, avrc, world: int, rank: int):
        """This rank's chains of a chained- (or reference-) model container
        (avr_decompress_chain_range): (lo, hi, status, regen, offsets, lens) for the plan's slices
        [lo, hi); status 0 regenerated, 1 not coded, < 0 failed."""
        return self._chain_range(lib().avr_decompress_chain_range, "decompress_chain_range", avrc, world, rank)

    def slice_kernel(self, n: int, max_mb_width: int, decompress: bool, p32: bool = False) -> str:
        """The kernel a parallel-model batch of n slices runs (avr_slice_kernel), named as rocprofv3
        reports it: slices_parallel_kernel (resident) or slices_queue_kernel (persistent queue),
        template <MODE, FLD = false, P32>."""
        k = ctypes.c_int(-1)
        self._check(lib().avr_slice_kernel(self._h, 1 if decompress else 0, n, max_mb_width, ctypes.byref(k)),
                    "slice_kernel")
        name = ("slices_parallel_kernel", "slices_queue_kernel")[k.value]
        return f"{name}<{1 if decompress else 0}, false, {'true' if p32 else 'false'}>"

    def pack_outputs(self, d_desc, d_res, n, d_out, d_packed, d_offsets, stream=None):
        P = self._ptr
        self._check(lib().avr_pack_outputs(self._h, P(d_desc), P(d_res), n, P(d_out), P(d_packed), P(d_offsets),
                                           self._stream(stream)), "pack_outputs")

    # ------------------------------------------------------------------ synthetic input
    def synthesize(self, params: SynthParams, n: int) -> bytes:
        sp = _SynthParams(params.mb_width, params.mb_height, params.slice_type, params.slice_qp,
                          params.chroma_format_idc, params.transform_8x8_mode, params.num_ref_idx_l0,
                          params.num_ref_idx_l1, params.seed, params.slices_per_picture, params.gop_length,
                          params.repeat, params.structure)
        out, olen = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(lib().avr_synthesize_stream(self._h, ctypes.byref(sp), int(n), ctypes.byref(out),
                                                ctypes.byref(olen)), "synthesize")
        return _take(out, olen.value)
