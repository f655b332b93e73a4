"""Batch roundtrip diagnosis (experiment tool): a synthetic 1080p I-slice batch through the device
roundtrip; for slices that do not verify: compress / decompress statuses and lengths, and the
oracle's per-slice result for the first few of them."""
import argparse
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import numpy as np
import torch
import avrecode_amd as avr
from avrecode_amd.batch import DeviceBatch
import bench
import _oracle

n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
args = argparse.Namespace(mb_width=120, mb_height=68, seed=0)
with avr.Context(0) as ctx:
    data = bench.make_input(ctx, n, 0, args)
    ps = avr.parse_stream(data)
    b = DeviceBatch(ctx, ps)
    b.roundtrip(avr.MODEL_PARALLEL)
    torch.cuda.synchronize()
    v, rc, rd = b.verdicts(), b.results("c"), b.results("d")
    rec, regen, pays = b.recoded(), b.regenerated(), b.payloads()
bad = np.nonzero(v != 1)[0]
print(f"{n} slices, {len(bad)} not verified: {bad[:40].tolist()}")
for k in bad[:3]:
    k = int(k)
    dv = rec[k]
    la = int.from_bytes(dv[:4], "little") if len(dv) >= 4 else -1
    rg, pay = regen[k], pays[k]
    fd = next((i for i in range(min(len(rg), len(pay))) if rg[i] != pay[i]), None)
    print(f"slice {k}: st_c {rc[k]['status']} len_c {rc[k]['out_len']} lenA {la} cap {ps.descs[k]['out_capacity']} "
          f"bins_c {rc[k]['bins']} | st_d {rd[k]['status']} len_d {rd[k]['out_len']} bins_d {rd[k]['bins']} "
          f"payload {len(pay)} first regen diff {fd}")
    _, ref = _oracle.slices_p(data, k, k + 1)
    r = ref[0]
    orc = r["recoded"]
    first = next((i for i in range(min(len(dv), len(orc))) if dv[i] != orc[i]), None)
    print(f"   oracle: st_c {r['status_c']} bins {r['bins']} len {len(orc)} lenA {int.from_bytes(orc[:4], 'little')} "
          f"device==oracle {dv == orc} first diff {first}; oracle regen ok {_oracle.patch_restores(r['regen'], pay)}")
