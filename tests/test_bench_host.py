"""bench.py host logic (no GPU): the all-cores CPU baseline cuts one synthesized Annex-B stream into
standalone single-slice files (the stream's parameter sets + one slice NAL unit each).  A slice of
the parallel model is independent of its neighbours, so the oracle must give each standalone file
exactly what it gives that slice inside the whole stream -- otherwise the baseline would time
different work than the batch it stands for."""
import sys

from _oracle import ROOT, build_oracle, slices_p

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_split_slices_layout():
    s = (b"\x00\x00\x00\x01\x67SPS" + b"\x00\x00\x00\x01\x68PPS" + b"\x00\x00\x01\x65IDR\x01"
         + b"\x00\x00\x00\x00\x01\x41P\x80" + b"\x00\x00\x01\x06SEI")
    head, nals = bench._split_slices(s)
    assert head == b"\x00\x00\x00\x01\x67SPS\x00\x00\x00\x01\x68PPS"
    # trailing zero bytes before a start code are not part of the NAL unit; an SEI after the
    # first slice is neither a slice nor part of the parameter-set head
    assert nals == [b"\x00\x00\x00\x01\x65IDR\x01", b"\x00\x00\x00\x01\x41P\x80"]


def test_standalone_slices_match_the_stream():
    build_oracle()
    data = (ROOT / "tests" / "fixtures" / "paff_ipp.264").read_bytes()
    head, nals = bench._split_slices(data)
    total, whole = slices_p(data, 0, 4)
    assert total == len(nals) and len(whole) == 4
    for i in range(4):
        n, one = slices_p(head + nals[i], 0, 1)
        assert n == 1
        assert one[0]["status_c"] == whole[i]["status_c"] == 0
        assert one[0]["bins"] == whole[i]["bins"]
        assert one[0]["recoded"] == whole[i]["recoded"]
        assert one[0]["regen"] == whole[i]["regen"]


def test_bench_golden_is_consistent():
    """tests/golden/bench_batch.json (the oracle's answer for the headline batch, made by
    tests/golden/make_bench_golden.py): one record per slice, totals equal to the sums, every slice
    coded by the oracle; bench.golden_check applies it only to the batch it was made for."""
    import json

    import bench
    g = json.loads(bench.GOLDEN_BATCH.read_text())
    assert g["config"]["slices"] == len(g["slices"]) == 1024 and g["config"]["seed"] == 0
    assert g["bins_total"] == sum(s["bins"] for s in g["slices"])
    assert g["recoded_total"] == sum(s["recoded_len"] for s in g["slices"])
    assert all(s["status"] == 0 and len(s["recoded_sha256"]) == 64 for s in g["slices"])

    class A:
        slices, mb_width, mb_height, seed = 1024, 120, 68, 1
    assert bench.golden_check(None, b"", A) is None   # another seed: not this golden's batch
