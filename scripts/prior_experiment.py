"""does a per-file prior for the parallel model's per-context estimators make
its containers smaller than the input?  CPU only, on the oracle (test infrastructure).

For each file: the oracle's P-mode and R-mode containers; then a first pass counting every coded
bin of a per-context (default) key by context and value (AVR_ORACLE_STATS); then P-mode with
every per-context estimator starting from the file's own frequencies at a few strengths S (pos + neg
= S, each >= 1; AVR_ORACLE_PRIOR).  The prior would travel in the container: its cost is counted as
2 bytes per context the file uses (context index implied by a bitmap: 1026 bits) added to the
container.  Writes a JSON report.

  python scripts/prior_experiment.py OUT.json FILE...
"""
import json
import os
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
from _oracle import build_oracle  # noqa: E402

STRENGTHS = (4, 8, 16, 32, 64)


def compress(cli, path, mode, env=None):
    with tempfile.TemporaryDirectory() as td:
        o = Path(td) / "o.avrc"
        args = [str(cli), "compress"] + {"R": [], "P": ["-p"]}[mode] + [str(path), str(o)]
        r = subprocess.run(args, capture_output=True, env=dict(os.environ, **(env or {})))
        if r.returncode != 0:
            raise RuntimeError(r.stderr.decode())
        return o.stat().st_size


def main():
    out, files = sys.argv[1], sys.argv[2:]
    _, cli = build_oracle()
    rep = []
    for f in files:
        n = os.path.getsize(f)
        row = {"file": os.path.basename(f), "bytes": n, "R": compress(cli, f, "R"), "P": compress(cli, f, "P")}
        with tempfile.TemporaryDirectory() as td:
            st = Path(td) / "stats.bin"
            compress(cli, f, "P", {"AVR_ORACLE_STATS": str(st)})
            c = np.frombuffer(st.read_bytes(), dtype=np.uint64).reshape(1026, 2).astype(np.float64)
            used = (c.sum(1) > 0)
            row["contexts_used"] = int(used.sum())
            cost = 2 * int(used.sum()) + 1026 // 8
            for S in STRENGTHS:
                p1 = (c[:, 1] + 0.5) / (c.sum(1) + 1.0)
                pos = np.clip(np.rint(p1 * S), 1, S - 1)
                neg = np.clip(S - pos, 1, S - 1)
                pr = np.zeros((1026, 2), np.uint16)
                pr[used, 0] = pos[used]
                pr[used, 1] = neg[used]
                pf = Path(td) / f"prior{S}.bin"
                pf.write_bytes(pr.tobytes())
                size = compress(cli, f, "P", {"AVR_ORACLE_PRIOR": str(pf)})
                row[f"P_prior{S}"] = size
                row[f"P_prior{S}_with_cost"] = size + cost
        row["ratio_R"] = row["R"] / n
        row["ratio_P"] = row["P"] / n
        best = min(STRENGTHS, key=lambda S: row[f"P_prior{S}_with_cost"])
        row["best_S"] = best
        row["ratio_P_best_prior"] = row[f"P_prior{best}_with_cost"] / n
        print(json.dumps(row), flush=True)
        rep.append(row)
    Path(out).write_text(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
