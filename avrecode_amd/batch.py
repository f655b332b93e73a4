"""Device-resident slice batches: HBM layout + one call per roundtrip (avr_roundtrip_slices).

HBM layout of a batch (DESIGN.md "Data layout"):
  d_in      payload arena: slice k's unescaped CABAC payload at desc[k].payload_offset (16-B aligned,
            >= 16 zero bytes after it) -- exactly what init_decoder receives (recode.cpp:143)
  d_work    re-coded output: slice k at desc[k].out_offset, desc[k].out_capacity bytes reserved
  d_regen   regenerated CABAC bytes, laid out like d_in
  d_desc / d_dec_desc   avr_slice_desc[n] (96 B each) for compress / derived decompress
  d_res_c / d_res_d     avr_slice_result[n] (40 B each); d_verdict int32[n]
torch only allocates and owns these buffers and supplies the stream; all compute is in
libavrecode.so.
"""
from __future__ import annotations

import numpy as np
import torch

from . import SLICE_DESC, SLICE_RESULT, MODEL_PARALLEL, Context, ParsedStream


def _dev_bytes(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(device)


class DeviceBatch:
    def __init__(self, ctx: Context, ps: ParsedStream, device=None):
        self.ctx = ctx
        self.ps = ps
        self.device = torch.device("cuda", ctx.device) if device is None else device
        self.n = len(ps.descs)
        n = max(1, self.n)
        self.d_desc = _dev_bytes(ps.descs, self.device)
        self.d_in = _dev_bytes(ps.arena, self.device)
        self.d_work = torch.zeros(max(16, ps.work_len + 16), dtype=torch.uint8, device=self.device)
        self.d_regen = torch.zeros_like(self.d_in)
        self.d_dec_desc = torch.zeros(n * SLICE_DESC.itemsize, dtype=torch.uint8, device=self.device)
        self.d_res_c = torch.zeros(n * SLICE_RESULT.itemsize, dtype=torch.uint8, device=self.device)
        self.d_res_d = torch.zeros_like(self.d_res_c)
        self.d_verdict = torch.zeros(n, dtype=torch.int32, device=self.device)

    def roundtrip(self, model: int = MODEL_PARALLEL, stream=None):
        self.ctx.roundtrip_slices(self.d_desc, self.n, self.ps.max_mb_width, self.ps.max_mb_height, self.d_in,
                                  self.d_work, self.d_regen, self.d_dec_desc, self.d_res_c, self.d_res_d,
                                  self.d_verdict, model, stream)

    def roundtrip_timed(self, ev, model: int = MODEL_PARALLEL, stream=None):
        """roundtrip() as its four launches; ev = 4 events recorded on `stream`:
        ev[0] compress ev[1] derive ev[2] decompress ev[3] verify."""
        c, n, w, h = self.ctx, self.n, self.ps.max_mb_width, self.ps.max_mb_height
        ev[0].record(stream)
        c.compress_slices(self.d_desc, n, w, h, self.d_in, self.d_work, self.d_res_c, model, stream)
        ev[1].record(stream)
        c.derive_decompress_descs(self.d_desc, self.d_res_c, n, self.d_dec_desc, stream)
        ev[2].record(stream)
        c.decompress_slices(self.d_dec_desc, n, w, h, self.d_work, self.d_regen, self.d_res_d, model, stream)
        ev[3].record(stream)
        c.verify_slices(self.d_desc, self.d_res_c, self.d_res_d, n, self.d_in, self.d_regen, self.d_verdict, stream)

    def compress(self, model: int = MODEL_PARALLEL, stream=None):
        self.ctx.compress_slices(self.d_desc, self.n, self.ps.max_mb_width, self.ps.max_mb_height, self.d_in,
                                 self.d_work, self.d_res_c, model, stream)

    def decompress(self, model: int = MODEL_PARALLEL, stream=None):
        """A decompress batch (ps from plan_decompress: payloads = re-coded streams): d_in -> d_work,
        results in d_res_d (avr_decompress_slices)."""
        self.ctx.decompress_slices(self.d_desc, self.n, self.ps.max_mb_width, self.ps.max_mb_height, self.d_in,
                                   self.d_work, self.d_res_d, model, stream)

    def pack(self, stream=None, which: str = "c"):
        """d_work's per-slice outputs packed contiguously on the device (avr_pack_outputs) by the
        compress ("c") or decompress ("d") results: (d_packed uint8, d_offsets uint64[n + 1]); slice
        k's bytes (status 0) start at offsets[k]."""
        if not hasattr(self, "d_packed"):
            self.d_packed = torch.zeros(max(16, self.ps.work_len + 16), dtype=torch.uint8, device=self.device)
            self.d_offsets = torch.zeros(max(1, self.n) + 1, dtype=torch.int64, device=self.device)
        res = self.d_res_c if which == "c" else self.d_res_d
        self.ctx.pack_outputs(self.d_desc, res, self.n, self.d_work, self.d_packed, self.d_offsets, stream)
        return self.d_packed, self.d_offsets

    # ----------------------------------------------------------------- results (host copies)
    def results(self, which: str = "c") -> np.ndarray:
        t = self.d_res_c if which == "c" else self.d_res_d
        return t.cpu().numpy().view(SLICE_RESULT)[: self.n]

    def verdicts(self) -> np.ndarray:
        return self.d_verdict.cpu().numpy()[: self.n]

    def recoded(self) -> list[bytes]:
        """Per-slice re-coded bytes (b'' where compress failed)."""
        res = self.results("c")
        work = self.d_work.cpu().numpy()
        out = []
        for k, d in enumerate(self.ps.descs):
            o, ln = int(d["out_offset"]), int(res[k]["out_len"])
            out.append(work[o:o + ln].tobytes() if res[k]["status"] == 0 and d["coded"] else b"")
        return out

    def regenerated(self) -> list[bytes]:
        res = self.results("d")
        regen = self.d_regen.cpu().numpy()
        out = []
        for k, d in enumerate(self.ps.descs):
            o, ln = int(d["payload_offset"]), int(res[k]["out_len"])
            out.append(regen[o:o + ln].tobytes() if res[k]["status"] == 0 else b"")
        return out

    def payloads(self) -> list[bytes]:
        return [self.ps.arena[int(d["payload_offset"]):int(d["payload_offset"]) + int(d["payload_size"])].tobytes()
                for d in self.ps.descs]


class DecompressRange:
    """One rank's decompress batch of a sharded container decompress, in device buffers that grow
    as needed and are reused from step to step: the planned slices' descriptors and re-coded
    streams (d_desc, d_in), the regenerated bytes (d_work), the results (d_res), and their packed
    copy (d_packed, d_offsets) for the gather to rank 0.  upload() takes a host ParsedStream
    (DecompressPlan.parsed / shard.subset) or device tensors received from rank 0."""

    def __init__(self, ctx: Context, device=None):
        self.ctx = ctx
        self.device = torch.device("cuda", ctx.device) if device is None else device
        self.n = 0
        self._cap = {}

    def _buf(self, name: str, nbytes: int, dtype=torch.uint8) -> torch.Tensor:
        itemsize = torch.empty(0, dtype=dtype).element_size()
        count = max(1, (nbytes + itemsize - 1) // itemsize)
        t = self._cap.get(name)
        if t is None or t.numel() < count:
            t = torch.empty(count + count // 16, dtype=dtype, device=self.device)
            self._cap[name] = t
        return t

    def upload(self, descs, arena, n: int, work_len: int, max_mb_width: int, max_mb_height: int, stream=None):
        """descs / arena: numpy (host) or uint8 torch tensors (device)."""
        self.n, self.work_len = n, work_len
        self.max_mb_width, self.max_mb_height = max_mb_width, max_mb_height
        nd = n * SLICE_DESC.itemsize
        self.d_desc = self._buf("desc", nd)
        self.d_in = self._buf("in", (arena.nbytes if isinstance(arena, np.ndarray) else arena.numel()) + 16)
        with torch.cuda.stream(stream) if stream is not None else _null():
            for dst, src, k in ((self.d_desc, descs, nd), (self.d_in, arena, None)):
                if isinstance(src, np.ndarray):
                    src = torch.from_numpy(np.ascontiguousarray(src).view(np.uint8).reshape(-1))
                k = src.numel() if k is None else k
                if k:
                    dst[:k].copy_(src[:k], non_blocking=False)
        self.d_work = self._buf("work", work_len + 16)
        self.d_res = self._buf("res", max(1, n) * SLICE_RESULT.itemsize)

    def run(self, model: int = MODEL_PARALLEL, stream=None):
        self.ctx.decompress_slices(self.d_desc, self.n, self.max_mb_width, self.max_mb_height, self.d_in, self.d_work,
                                   self.d_res, model, stream)

    def pack(self, stream=None):
        d_packed = self._buf("packed", self.work_len + 16)
        d_offsets = self._buf("offsets", 8 * (self.n + 1), torch.int64)
        self.ctx.pack_outputs(self.d_desc, self.d_res, self.n, self.d_work, d_packed, d_offsets, stream)
        return d_packed, d_offsets

    def results(self) -> np.ndarray:
        return self.d_res[:max(1, self.n) * SLICE_RESULT.itemsize].cpu().numpy().view(SLICE_RESULT)[: self.n]


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
