"""SQ / SQC counters per launch of the slice kernels from rocprofv3 PMC passes (scripts/pmc.sh),
summed over the kernel's dispatch, averaged over launches, and per CABAC bin of the launch's batch.

  python scripts/pmc_sq.py gpurun_out/pmc_<tag> profiles/<tag>_sq_counters.json --bins <bins per launch>
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# progressive-slice kernels of the u64 coder (template <MODE, FLD, P32> since round 4; the
# field-capable instantiations return at once on a progressive batch)
# (the resident kernel of the headline batch, the persistent queue kernel of the configs[3] stream)
KERNELS = {"slices_parallel_kernel<0, false, false>": "compress", "slices_parallel_kernel<1, false, false>": "decompress",
           "slices_queue_kernel<0, false, false>": "compress", "slices_queue_kernel<1, false, false>": "decompress"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--bins", type=int, required=True, help="CABAC bins per launch (bench config.bins)")
    a = ap.parse_args()
    # (kernel, counter) -> {dispatch id: summed value}
    vals = defaultdict(lambda: defaultdict(float))
    for p in glob.glob(os.path.join(a.src, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            name = next((v for k, v in KERNELS.items() if k in r["Kernel_Name"]), None)
            if name is None:
                continue
            vals[(name, r["Counter_Name"])][(p, r["Dispatch_Id"])] += float(r["Counter_Value"])
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from avrecode_amd import source_sha   # the build the counters were taken on
    out = {"source": a.src, "source_sha": source_sha(), "bins_per_launch": a.bins, "kernels": {}}
    for (name, ctr), d in sorted(vals.items()):
        per_launch = sum(d.values()) / len(d)
        k = out["kernels"].setdefault(name, {})
        k[ctr] = {"per_launch": per_launch, "per_bin": per_launch / a.bins, "launches": len(d)}
    for name, k in out["kernels"].items():
        salu, valu = k.get("SQ_INSTS_SALU", {}).get("per_bin"), k.get("SQ_INSTS_VALU", {}).get("per_bin")
        if salu is not None and valu is not None:
            k["summary_per_bin"] = {c.replace("SQ_INSTS_", ""): round(k[c]["per_bin"], 2)
                                    for c in ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS",
                                              "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR") if c in k}
        if "SQC_ICACHE_MISSES" in k and "SQC_ICACHE_HITS" in k:
            m, h = k["SQC_ICACHE_MISSES"]["per_launch"], k["SQC_ICACHE_HITS"]["per_launch"]
            k["icache_miss_rate"] = m / max(1.0, m + h)
    json.dump(out, open(a.dst, "w"), indent=1)
    print(json.dumps({n: k.get("summary_per_bin") for n, k in out["kernels"].items()}, indent=1))
    for n, k in out["kernels"].items():
        print(n, "icache miss rate", k.get("icache_miss_rate"),
              {c: round(k[c]["per_bin"], 1) for c in k if c.startswith("SQ_W") or c.startswith("SQ_A") or c == "SQ_BUSY_CYCLES"})


if __name__ == "__main__":
    main()
