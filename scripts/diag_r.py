"""R-mode / P-mode whole-file diagnosis (experiment tool): device containers vs the oracle's, and
device decompress of the oracle's containers, for the fixtures."""
import hashlib
import json
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import avrecode_amd as avr
from _oracle import oracle_cli

GOLD = {(g["file"], g["mode"]): g for g in json.loads((ROOT / "tests/golden/fixtures.json").read_text())}
with avr.Context(0) as ctx:
    for name in ("realshort.mp4", "cockatoo.mp4"):
        data = (ROOT / "tests" / "fixtures" / name).read_bytes()
        for mode, model in (("R", avr.MODEL_REFERENCE), ("P", avr.MODEL_PARALLEL)):
            ora = oracle_cli("compress", ROOT / "tests" / "fixtures" / name, mode=mode)
            try:
                dev = ctx.compress(data, model)
            except Exception as e:
                dev = b""
                print(name, mode, "compress raised", e)
            first = next((i for i in range(min(len(dev), len(ora))) if dev[i] != ora[i]), None)
            print(name, mode, "container dev == oracle:", dev == ora, "len", len(dev), len(ora), "first diff", first,
                  "golden:", hashlib.sha256(ora).hexdigest() == GOLD[(name, mode)]["avrc_sha256"])
            for tag, c in (("oracle", ora), ("device", dev)):
                try:
                    back = ctx.decompress(c)
                    fd = next((i for i in range(min(len(back), len(data))) if back[i] != data[i]), None)
                    print("   decompress of", tag, "container ok:", back == data, "len", len(back), "first diff", fd)
                except Exception as e:
                    print("   decompress of", tag, "container raised", e)
