"""HBM traffic per launch of the slice kernels from rocprofv3 PMC passes (scripts/pmc.sh).

  python scripts/pmc_traffic.py gpurun_out/pmc_<tag> profiles/<round>_pmc.json --slices 1024 --mb 120 68
  python scripts/pmc_traffic.py gpurun_out/pmc_<tag> profiles/<round>_stream_pmc.json --leg stream_shard \
      --seconds 600 --mb 240 135      (the configs[3] leg: bench.py --stream-shard)

FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB per dispatch (TCC_EA0_RDREQ/WRREQ
based).  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section), on gfx950 FETCH_SIZE counts
128-B read requests at 64 B, so it is doubled here; WRITE_SIZE is taken as reported.  The result
is what bench.py's roofline.traffic reads (bytes per launch, averaged over the dispatches).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# the progressive-slice kernels of the u64 coder, template <MODE, FLD, P32>: the resident kernel
# (the headline batch) and the persistent queue kernel (the configs[3] stream: thousands of 4K
# slices), as rocprofv3 names them (avrecode_amd.Context.slice_kernel)
KERNELS = tuple(f"{k}<{m}, false, false>" for k in ("slices_parallel_kernel", "slices_queue_kernel") for m in (0, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--slices", type=int, default=0)
    ap.add_argument("--mb", type=int, nargs=2, required=True)
    ap.add_argument("--leg", default="headline", help="headline (configs[2] batch) or stream_shard (configs[3])")
    ap.add_argument("--seconds", type=int, default=0, help="stream_shard: the stream's length")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for p in glob.glob(os.path.join(a.src, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            # the progressive-slice kernels of the u64 coder only (the field-capable instantiations
            # return at once on a progressive batch; the P32 ones are another container format)
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k is None:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from avrecode_amd import source_sha
    out = {"leg": a.leg, "slices": a.slices, "seconds": a.seconds, "mb": list(a.mb), "source": a.src,
           "source_sha": source_sha(),
           "note": "FETCH_SIZE x2 (gfx950 correction), WRITE_SIZE as reported; KiB -> bytes; mean per dispatch",
           "kernels": {}}
    for k, c in vals.items():
        fetch = 2 * 1024 * sum(c.get("FETCH_SIZE", [0])) / max(1, len(c.get("FETCH_SIZE", [])))
        write = 1024 * sum(c.get("WRITE_SIZE", [0])) / max(1, len(c.get("WRITE_SIZE", [])))
        out["kernels"][k] = {"fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                             "hbm_bytes_per_launch": fetch + write}
    json.dump(out, open(a.dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
