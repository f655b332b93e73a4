"""Chain length of the chained reference model (oracle, CPU only; experiment tool): for each file
and chain length k (AVR_ORACLE_CHAIN=k, the oracle's override of AVR_CHAIN_SLICES), the container's
size over the input and the number of chains (the decompress parallelism); every container is
decompressed back with the same k ("chains" counts ceil(parsed slices / k), an upper bound on the
coded chains).  k = 1 is the parallel model's blocks, k past the slice count
the reference model's.

  python scripts/chain_experiment.py OUT.json FILE...
"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
from _oracle import build_oracle  # noqa: E402

KS = (1, 2, 4, 8, 16, 32, 64, 1 << 30)


def main():
    out, files = sys.argv[1], sys.argv[2:]
    _, cli = build_oracle()
    rep = []
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            n = os.path.getsize(f)
            row = {"file": os.path.basename(f), "bytes": n}
            for mode, flag in (("R", []), ("P", ["-p"])):
                o = Path(td) / "o.avrc"
                subprocess.run([str(cli), "compress"] + flag + [f, str(o)], check=True, capture_output=True)
                row[mode] = o.stat().st_size / n
            for k in KS:
                env = dict(os.environ, AVR_ORACLE_CHAIN=str(k))
                o, back = Path(td) / "c.avrc", Path(td) / "c.out"
                subprocess.run([str(cli), "compress", "-c", f, str(o)], check=True, capture_output=True, env=env)
                subprocess.run([str(cli), "decompress", str(o), str(back)], check=True, capture_output=True, env=env)
                assert back.read_bytes() == Path(f).read_bytes(), (f, k)
                r = subprocess.run([str(cli), "slices", f], capture_output=True, text=True)
                coded = int(r.stdout.split("slices ok ")[1].split()[0])
                row[f"C{k if k < (1 << 30) else 'inf'}"] = {"ratio": o.stat().st_size / n, "chains": -(-coded // k)}
            print(json.dumps(row), flush=True)
            rep.append(row)
    Path(out).write_text(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
