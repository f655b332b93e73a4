"""Debug helper: MBAFF / PAFF synthetic streams, device P-mode roundtrip verdicts, streams saved
under gpurun_out/ for the CPU oracle."""
import json, os, sys
sys.path.insert(0, '.')
import torch
import avrecode_amd as avr
from avrecode_amd.batch import DeviceBatch
ctx = avr.Context(0)
out = {}
cases = {
    "m_i": dict(slice_type=2, transform_8x8_mode=0),
    "m_i8": dict(slice_type=2, transform_8x8_mode=1),
    "m_p": dict(slice_type=0, transform_8x8_mode=0, gop_length=2),
    "m_p8": dict(slice_type=0, transform_8x8_mode=1, gop_length=3, num_ref_idx_l0=2),
    "m_b": dict(slice_type=1, transform_8x8_mode=1, gop_length=4, num_ref_idx_l0=2, num_ref_idx_l1=2),
    "m_422": dict(slice_type=0, chroma_format_idc=2, gop_length=2),
    "m_444": dict(slice_type=1, chroma_format_idc=3, gop_length=3),
    "m_spp": dict(slice_type=0, gop_length=2, slices_per_picture=3),
}
for name, kw in cases.items():
    args = dict(mb_width=11, mb_height=8, slice_qp=27, seed=3, structure=2); args.update(kw)
    data = ctx.synthesize(avr.SynthParams(**args), 2)
    open(f"gpurun_out/{name}.264", "wb").write(data)
    ps = avr.parse_stream(data)
    b = DeviceBatch(ctx, ps); b.roundtrip(avr.MODEL_PARALLEL); torch.cuda.synchronize()
    out[name] = dict(verdict=[int(x) for x in b.verdicts()], status=[int(x) for x in b.results("c")["status"]],
                     dstatus=[int(x) for x in b.results("d")["status"]], bins=[int(x) for x in b.results("c")["bins"]])
    print(name, json.dumps(out[name]), flush=True)
