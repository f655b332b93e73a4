"""Debug helper: synthesize one stream, save it and the device's R / P containers (and the
sequential R-mode one) under gpurun_out/ for CPU-side comparison with the oracle."""
import json, os, sys
sys.path.insert(0, '.')
import avrecode_amd as avr
ctx = avr.Context(0)
kw = json.loads(sys.argv[2])
name = sys.argv[1]
n = int(kw.pop("n", 4))
data = ctx.synthesize(avr.SynthParams(**kw), n)
open(f"gpurun_out/{name}.264", "wb").write(data)
open(f"gpurun_out/{name}.R.avrc", "wb").write(ctx.compress(data, avr.MODEL_REFERENCE))
open(f"gpurun_out/{name}.P.avrc", "wb").write(ctx.compress(data, avr.MODEL_PARALLEL))
os.environ["AVR_RMODE_SEQUENTIAL"] = "1"
open(f"gpurun_out/{name}.Rseq.avrc", "wb").write(ctx.compress(data, avr.MODEL_REFERENCE))
print("ok", name, len(data))
