"""bench.py's N > 1 code paths, executed before the driver's multi-GPU run meets them.

`python -m torch.distributed.run --nproc-per-node 2 bench.py --gpus 2 ...` exactly as the driver
launches it, at tiny sizes, with the collectives on gloo (AVR_DIST_BACKEND=gloo: both ranks share
this box's one GPU, and RCCL will not put two ranks on one device):
* the default mode: every rank's weak-scaling batch (headline), the max-over-ranks reduction, the
  corpus dealt over the ranks (corpus_sharded);
* --stream-shard (BASELINE configs[3]): the stream cut over the ranks, the gather to rank 0 and its
  container assembly, rank 0's plan of that container scattered over the ranks, every rank's
  decompress, the gather of the regenerated slices and rank 0's splice into the stream.
Each run must print one JSON line with n_gpus 2 and bit_exact true.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from _oracle import ROOT

pytestmark = pytest.mark.gpu


def _run_two_ranks(extra):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, AVR_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_default_mode_two_ranks():
    line = _run_two_ranks(["--steps", "1", "--warmup", "1", "--slices", "8", "--mb-width", "40", "--mb-height", "24",
                           "--corpus-scale", "0.05", "--stream-leg-seconds", "1", "--stream-mb", "20", "12"])
    assert line["n_gpus"] == 2 and line["bit_exact"] is True
    assert line["scaling"] == "weak" and line["value"] > 0
    assert line["corpus"]["n_gpus"] == 2
    assert all(line["corpus"][m]["bit_exact"] is True for m in ("R", "P", "C"))
    assert "chains" in line["corpus"]["C_split"]   # C: each file's chains over both ranks
    # the configs[3] leg sharded over both ranks inside the default run
    st = line["stream_shard"]
    assert st["n_gpus"] == 2 and st["bit_exact"] is True and st["config"]["slices"] == 30
    _check_setup_scales(st)


def _check_setup_scales(line):
    """Rank 0 parses the whole stream (its assembly reads every slice); rank 1 holds only its own
    range's descriptors and payload bytes (setup work on ranks > 0 ~ 1/N)."""
    r0, r1 = line["config"]["setup_by_rank"]
    n = line["config"]["slices"]
    assert r0["slices_parsed"] == n and 0 < r1["slices_parsed"] < n
    assert r1["payload_bytes_copied"] < 0.8 * r0["payload_bytes_copied"]


def test_bench_stream_shard_two_ranks():
    line = _run_two_ranks(["--stream-shard", "--stream-seconds", "1", "--stream-mb", "20", "12", "--steps", "1",
                           "--warmup", "1"])
    assert line["n_gpus"] == 2 and line["bit_exact"] is True
    assert line["scaling"] == "strong" and line["config"]["slices"] == 30
    assert set(line["config"]["step_phases_s_rank0"]) == {
        "compress_s", "results_d2h_s", "gather_s", "assemble_s", "plan_s", "scatter_h2d_s", "decompress_s",
        "gather_d_s", "splice_s"}
    _check_setup_scales(line)
